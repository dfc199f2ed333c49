#!/bin/bash
# A/B of expand_fast's probe rounds: SR_PROBE_BATCH=1 (default) against 3 (one round of lookahead:
# the next successor's probe load issued before the current one is resolved). Parity first (the
# FAST-order GPU parity tests with the pipelined kernel forced on), then alternating bench runs.
#   scripts/gpu_pipe_ab.sh <tag>
set -o pipefail
TAG=${1:?tag}
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$TAG
mkdir -p "$O"
SR_PROBE_BATCH=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > "$O/parity_pb3.log" 2>&1 || { tail -30 "$O/parity_pb3.log"; exit 1; }
tail -1 "$O/parity_pb3.log"
run() {  # run <pb> <label> <bench args...>
    local pb=$1 label=$2; shift 2
    SR_PROBE_BATCH=$pb timeout -k 10 200 python -u bench.py --cpu-baseline 0 --config4-steps 0 --no-hint-steps 0 "$@" > "$O/$label.json" 2> "$O/$label.err" || { tail -5 "$O/$label.err"; return 1; }
    python3 -c "import json,sys; d=json.loads(open('$O/$label.json').read().strip().splitlines()[-1]); l=d.get('levels',{}); print('$label', round(d['ms_per_step'],4), 'big', round(l.get('big_levels_ms',0),4), 'small', round(l.get('small_levels_ms',0),4))"
}
for r in 1 2; do
    run 1 "pb1_2pc9_$r" --steps 20 || exit 1
    run 3 "pb3_2pc9_$r" --steps 20 || exit 1
done
run 1 pb1_2pc10 --rm-count 10 --steps 5 || exit 1
run 3 pb3_2pc10 --rm-count 10 --steps 5 || exit 1
run 1 pb1_inclock10 --model increment_lock --threads 10 --steps 5 || exit 1
run 3 pb3_inclock10 --model increment_lock --threads 10 --steps 5 || exit 1
run 1 pb1_paxos3 --model paxos --steps 10 || exit 1
run 3 pb3_paxos3 --model paxos --steps 10 || exit 1
echo "ab ok"
