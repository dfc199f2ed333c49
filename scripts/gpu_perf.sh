# Bench 2pc/paxos + per-level traces (no test suite).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-baseline 0 2>/dev/null || exit 1
timeout -k 10 300 python bench.py --model paxos --steps 10 --warmup 3 --cpu-baseline 0 2>/dev/null || exit 1
bash scripts/ktrace.sh kt_2pc --steps 1 --warmup 1 --cpu-baseline 0 && bash scripts/ktrace.sh kt_paxos --model paxos --steps 1 --warmup 1 --cpu-baseline 0
