#!/bin/bash
# Round measurements on one MI355X (run through gpurun from the repo root):
#   scripts/gpu_round.sh <round tag, e.g. r02> [tests|bench|prof|pmc|all]
# Every GPU step has its own time limit and the steps stop at the first failure. Outputs land
# under gpurun_out/<tag>/; the files worth keeping are copied to profiles/<tag>_* by hand.
#   tests: the full `-m gpu` suite (log)
#   bench: the default bench line (2pc N=9 + config4 + cpu_baseline) and the side configs
#   prof : rocprofv3 --kernel-trace --stats of the default bench, and its per-level trace
#   pmc  : beyond-L2 traffic of expand_fast (scripts/pmc_traffic.sh, separate counter passes)
set -o pipefail
TAG=${1:?round tag}
WHAT=${2:-all}
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$TAG
mkdir -p "$O"
want() { [ "$WHAT" = all ] || [ "$WHAT" = "$1" ]; }
b() {
    local name=$1; shift
    timeout -k 10 300 python -u bench.py "$@" > "$O/$name.json" 2> "$O/$name.err" || { echo "bench $name failed"; tail -20 "$O/$name.err"; return 1; }
    tail -1 "$O/$name.json"
}

if want tests; then
    timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/gpu_tests.log" 2>&1 || { tail -40 "$O/gpu_tests.log"; exit 1; }
    tail -2 "$O/gpu_tests.log"
fi
if want bench; then
    b bench --steps 20 --warmup 3 || exit 1
    b bench_rccl1 --mode rccl1 --steps 10 --warmup 3 --cpu-baseline 0 --config4-steps 0 || exit 1
    b bench_2pc10 --rm-count 10 --steps 3 --warmup 1 --cpu-baseline 0 --config4-steps 0 || exit 1
    b bench_inclock11 --model increment_lock --threads 11 --steps 2 --warmup 1 --cpu-baseline 0 --config4-steps 0 || exit 1
    b bench_paxos3 --model paxos --clients 3 --steps 10 --warmup 3 --cpu-baseline 1 --config4-steps 0 || exit 1
    b bench_paxos6 --model paxos --clients 6 --steps 3 --warmup 1 --cpu-baseline 0 --config4-steps 0 || exit 1
    b bench_2pc11 --rm-count 11 --steps 2 --warmup 1 --cpu-baseline 0 --config4-steps 0 --no-hint-steps 0 || exit 1
    b bench_single_copy4 --model single_copy --clients 4 --steps 10 --warmup 3 --cpu-baseline 1 --config4-steps 0 || exit 1
fi
if want prof; then
    export TMPDIR=/tmp
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o bench -- python3 bench.py --steps 5 --warmup 2 --cpu-baseline 0 --config4-steps 0 > "$O/prof.log" 2>&1 || { echo "rocprof failed"; tail -20 "$O/prof.log"; exit 1; }
    tail -1 "$O/prof.log"
    bash scripts/ktrace.sh "$TAG/kt_2pc" --steps 1 --warmup 1 --cpu-baseline 0 --config4-steps 0 || exit 1
    python3 scripts/ktrace_levels.py "$O/kt_2pc/trace_kernel_trace.csv"
fi
if want pmc; then
    bash scripts/pmc_traffic.sh || exit 1
fi
