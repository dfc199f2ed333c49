#!/bin/bash
# Small levels at the start of a check in one workgroup (launch_tiny; SR_TINY=0 off, SR_TINY_SUCC the
# successor budget per level): the whole GPU suite, then ms per check, alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-q}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
run() {  # label env -- bench args
    local label=$1; shift
    local envs=()
    while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
    env "${envs[@]}" timeout -k 10 200 python -u bench.py --cpu-baseline 0 --config4-steps 0 --no-hint-steps 0 "$@" > "$O/$label.json" 2> "$O/$label.err" || { tail -5 "$O/$label.err"; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/$label.json').read().strip().splitlines()[-1]); l=d.get('levels') or {}; print('$label', round(d['ms_per_step'],4), 'small', round(l.get('small_levels_ms',0),4), 'big', round(l.get('big_levels_ms',0),4), 'launches', len(l.get('kernel_us') or []))"
}
for r in 1 2; do
    for e in "SR_TINY=0" "SR_TINY_SUCC=512" "SR_TINY_SUCC=1024" "SR_TINY_SUCC=2048"; do
        tag=$(echo $e | tr '=' '_')
        run px3_${tag}_r$r $e -- --model paxos --clients 3 --steps 200 --warmup 5 || exit 1
        run tp9_${tag}_r$r $e -- --steps 50 --warmup 3 || exit 1
    done
done
echo "quick ab ok"
