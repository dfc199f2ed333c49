set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_2pc9.json 2> gpurun_out/bench_2pc9.err || exit 1
cat gpurun_out/bench_2pc9.json
timeout -k 10 300 python bench.py --model paxos --clients 3 --steps 5 --warmup 2 > gpurun_out/bench_paxos3.json 2> gpurun_out/bench_paxos3.err || exit 1
cat gpurun_out/bench_paxos3.json
timeout -k 10 300 python bench.py --model paxos --clients 3 --order fifo --steps 5 --warmup 2 --cpu-baseline 0 > gpurun_out/bench_paxos3_fifo.json 2>&1 || exit 1
cat gpurun_out/bench_paxos3_fifo.json
