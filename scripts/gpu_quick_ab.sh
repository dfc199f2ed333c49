#!/bin/bash
# The visited set as ordinary (SR_TABLE_KIND=0), fine-grained (1) and uncached (2) device memory: does a
# kernel boundary after a big level cost the write-back of the L2s' dirty table lines?
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-q}
O=gpurun_out/$T
mkdir -p $O
SR_TABLE_KIND=2 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/parity_uc.log 2>&1 || { tail -30 $O/parity_uc.log; exit 1; }
tail -1 $O/parity_uc.log
run() {  # label env -- bench args
    local label=$1; shift
    local envs=()
    while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
    env "${envs[@]}" timeout -k 10 200 python -u bench.py --cpu-baseline 0 --config4-steps 0 --no-hint-steps 0 "$@" > "$O/$label.json" 2> "$O/$label.err" || { tail -5 "$O/$label.err"; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/$label.json').read().strip().splitlines()[-1]); l=d.get('levels') or {}; print('$label', round(d['ms_per_step'],4), 'small', round(l.get('small_levels_ms',0),4), 'big', round(l.get('big_levels_ms',0),4), 'gaps', round(l.get('gaps_ms',0),4))"
}
for r in 1 2; do
    for cfg in "tp9:--steps 50 --warmup 3" "tp10:--rm-count 10 --steps 5 --warmup 1" "px3:--model paxos --clients 3 --steps 200 --warmup 5"; do
        name=${cfg%%:*}; args=${cfg#*:}
        run ${name}_k0_r$r SR_TABLE_KIND=0 -- $args || exit 1
        run ${name}_k2_r$r SR_TABLE_KIND=2 -- $args || exit 1
        run ${name}_k1_r$r SR_TABLE_KIND=1 -- $args || exit 1
    done
done
SR_TABLE_KIND=2 bash scripts/ktrace.sh $T/kt_tp9_k2 --steps 20 --warmup 3 --cpu-baseline 0 --config4-steps 0 --no-hint-steps 0 || exit 1
echo "quick ab ok"
