#!/bin/bash
# Round 6: growth steps of unhinted checks after growth by ranges (SR_GROW_FIRST / SR_GROW_STEP),
# bench.py's no_hint line for 2pc N=9, N=10 and increment_lock N=11.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06gs
mkdir -p "$O"
for r in 1 2; do
  for e in "SR_X=0" "SR_GROW_FIRST=16" "SR_GROW_FIRST=32" "SR_GROW_STEP=16"; do
    for args in "--rm-count 9 --no-hint-steps 10" "--rm-count 10 --no-hint-steps 4" "--model increment_lock --threads 11 --no-hint-steps 2"; do
      tag=$(echo "$args" | tr -d ' -' | cut -c1-12)
      env $e timeout -k 10 200 python -u bench.py --cpu-baseline 0 --config4-steps 0 --steps 1 --warmup 1 $args \
          > "$O/${tag}_${e}_$r.json" 2> "$O/${tag}_${e}_$r.err" || { tail -5 "$O/${tag}_${e}_$r.err"; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/${tag}_${e}_$r.json').read().strip().splitlines()[-1]); n=d['no_hint']; print('$e r$r $args', 'no_hint', round(n['ms_per_step'],3), 'rehashes', n['rehashes'], 'cap', n['table_capacity'])"
    done
  done
done
echo "grow step ok"
