# Round measurements: bench lines (2pc N=9 default + larger configs + side models), rocprofv3
# kernel stats of the default bench, per-level kernel trace. Outputs under gpurun_out/meas/.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/meas
O=gpurun_out/meas
b() { local name=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$name.json 2> $O/$name.err && tail -1 $O/$name.json; }
b bench_2pc9 --steps 10 --warmup 3 || exit 1
b bench_2pc9_rccl1 --mode rccl1 --steps 10 --warmup 3 --cpu-baseline 0 || exit 1
b bench_2pc10 --rm-count 10 --steps 3 --warmup 1 --cpu-baseline 0 || exit 1
b bench_2pc11 --rm-count 11 --steps 2 --warmup 1 --cpu-baseline 0 || exit 1
b bench_inclock10 --model increment_lock --threads 10 --steps 3 --warmup 1 --cpu-baseline 0 || exit 1
b bench_inclock11 --model increment_lock --threads 11 --steps 2 --warmup 1 --cpu-baseline 0 || exit 1
b bench_paxos3 --model paxos --steps 10 --warmup 3 || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --steps 5 --warmup 2 --cpu-baseline 0 > $O/prof.log 2>&1 || exit 1
bash scripts/ktrace.sh meas/kt_2pc --steps 1 --warmup 1 --cpu-baseline 0 || exit 1
python3 scripts/ktrace_levels.py $O/kt_2pc/trace_kernel_trace.csv
