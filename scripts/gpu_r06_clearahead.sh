#!/bin/bash
# Round 6: clear-ahead (SR_CLEAR_AHEAD = 1 with 64 or 16 clearing workgroups / 0): the table-recycling tests, then back-to-back hinted
# checks of 2pc N=9, N=11, increment_lock N=11 and paxos C=3.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06ca
mkdir -p "$O"
timeout -k 10 400 python -u -m pytest tests/test_gpu_table_recycle.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
    -k "recycle or rehash or grow or closed_form or golden" > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
tail -2 "$O/tests.log"
for r in 1 2; do
  for e in "SR_CLEAR_BLOCKS=64" "SR_CLEAR_AHEAD=0" "SR_CLEAR_BLOCKS=16"; do
    for args in "--steps 20" "--rm-count 11 --steps 3 --warmup 1" "--model increment_lock --threads 11 --steps 4 --warmup 1" "--model paxos --clients 3 --steps 20"; do
      tag=$(echo "$args" | tr -d ' -' | cut -c1-20)
      env $e timeout -k 10 200 python -u bench.py --cpu-baseline 0 --config4-steps 0 --no-hint-steps 0 $args \
          > "$O/${tag}_${e}_r$r.json" 2> "$O/${tag}_${e}_r$r.err" || { tail -5 "$O/${tag}_${e}_r$r.err"; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/${tag}_${e}_r$r.json').read().strip().splitlines()[-1]); l=d.get('levels') or {}; print('$e r$r $args', round(d['ms_per_step'],4), 'span', round(l.get('span_ms',0),4))"
    done
  done
done
echo "clear-ahead ab ok"
