#!/bin/bash
# Verification pass at the current sources: the whole -m gpu suite, then bench lines of the
# headline and the side configurations. Every GPU step under its own limit; stops at the first
# failure. Usage: scripts/gpu_verify.sh <tag> [tests|bench|all]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:?tag}; WHAT=${2:-all}
O=gpurun_out/$T
mkdir -p $O
want() { [ "$WHAT" = all ] || [ "$WHAT" = "$1" ]; }
b() {
    local name=$1; shift
    timeout -k 10 300 python -u bench.py "$@" > "$O/$name.json" 2> "$O/$name.err" || { echo "bench $name failed"; tail -20 "$O/$name.err"; return 1; }
    python3 -c "import json,sys; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); l=d.get('levels') or {}; print('$name', round(d['ms_per_step'],4), 'ms', 'big', round(l.get('big_levels_ms') or 0,4), 'small', round(l.get('small_levels_ms') or 0,4), 'gaps', round(l.get('gaps_ms') or 0,4))"
}
if want tests; then
    timeout -k 10 1150 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/gpu_tests.log" 2>&1 || { tail -40 "$O/gpu_tests.log"; exit 1; }
    tail -2 "$O/gpu_tests.log"
fi
if want bench; then
    b bench9 --steps 20 --warmup 3 --cpu-baseline 0 --config4-steps 0 --no-hint-steps 0 || exit 1
    b bench10 --rm-count 10 --steps 3 --warmup 1 --cpu-baseline 0 --config4-steps 0 --no-hint-steps 0 || exit 1
    b bench11 --rm-count 11 --steps 2 --warmup 1 --cpu-baseline 0 --config4-steps 0 --no-hint-steps 0 || exit 1
    b paxos3 --model paxos --clients 3 --steps 10 --warmup 2 --cpu-baseline 0 --config4-steps 0 --no-hint-steps 0 || exit 1
    b paxos6 --model paxos --clients 6 --steps 5 --warmup 1 --cpu-baseline 0 --config4-steps 0 --no-hint-steps 0 || exit 1
    b single_copy4 --model single_copy --clients 4 --steps 10 --warmup 2 --cpu-baseline 0 --config4-steps 0 --no-hint-steps 0 || exit 1
    b inclock11 --model increment_lock --threads 11 --steps 3 --warmup 1 --cpu-baseline 0 --config4-steps 0 --no-hint-steps 0 || exit 1
fi
