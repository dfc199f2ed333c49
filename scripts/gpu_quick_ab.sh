#!/bin/bash
# The visited set in ordinary (SR_TABLE_KIND=0) or uncached (2) device memory for big tables: 2pc N=10 / N=11
# and increment_lock N=11 (quotient table, CAS-bound), alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-q}
O=gpurun_out/$T
mkdir -p $O
run() {  # label env -- bench args
    local label=$1; shift
    local envs=()
    while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
    env "${envs[@]}" timeout -k 10 200 python -u bench.py --cpu-baseline 0 --config4-steps 0 --no-hint-steps 0 "$@" > "$O/$label.json" 2> "$O/$label.err" || { tail -5 "$O/$label.err"; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/$label.json').read().strip().splitlines()[-1]); l=d.get('levels') or {}; print('$label', round(d['ms_per_step'],4), 'small', round(l.get('small_levels_ms',0),4), 'big', round(l.get('big_levels_ms',0),4))"
}
for r in 1 2; do
    for k in 0 2; do
        run tp10_k${k}_r$r SR_TABLE_KIND=$k -- --rm-count 10 --steps 5 --warmup 1 || exit 1
        run tp11_k${k}_r$r SR_TABLE_KIND=$k -- --rm-count 11 --steps 2 --warmup 1 || exit 1
        run il11_k${k}_r$r SR_TABLE_KIND=$k -- --model increment_lock --threads 11 --steps 3 --warmup 1 || exit 1
    done
done
echo "quick ab ok"
