# One GPU call: parity tests, the BASELINE bench, its rocprofv3 kernel-trace summary, side benches.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_2pc9.json 2> gpurun_out/bench_2pc9.err || exit 1
cat gpurun_out/bench_2pc9.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_2pc9 -o run -- python3 bench.py --steps 10 --warmup 3 --cpu-baseline 0 > gpurun_out/prof_2pc9.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --model paxos --clients 3 --steps 10 --warmup 3 > gpurun_out/bench_paxos3.json 2> gpurun_out/bench_paxos3.err || exit 1
cat gpurun_out/bench_paxos3.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_paxos3 -o run -- python3 bench.py --model paxos --clients 3 --steps 10 --warmup 3 --cpu-baseline 0 > gpurun_out/prof_paxos3.log 2>&1 || exit 1
find gpurun_out/prof_2pc9 gpurun_out/prof_paxos3 -name '*kernel_stats.csv'
