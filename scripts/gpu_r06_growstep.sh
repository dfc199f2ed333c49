#!/bin/bash
# Round 6: the growth step of an unhinted visited set (SR_GROW_STEP, default 8) on increment_lock N=11
# and 2pc N=9 / N=10 without capacity_hint.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06gs
mkdir -p $O
for e in "SR_GROW_STEP=8" "SR_GROW_STEP=16" "SR_GROW_STEP=32"; do
  env $e timeout -k 10 300 python -u bench.py --cpu-baseline 0 --config4-steps 0 --model increment_lock --threads 11 --steps 3 --warmup 1 --no-hint-steps 3 > $O/il11_${e#*=}.json 2> $O/il11_${e#*=}.err || { tail -5 $O/il11_${e#*=}.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/il11_${e#*=}.json').read().strip().splitlines()[-1]); n=d['no_hint']; print('inclock11 [$e] hinted', round(d['ms_per_step'],3), 'no_hint', round(n['ms_per_step'],3), 'vs', round(n['vs_value'],3), 'rehashes', n.get('rehashes'), 'cap', n.get('table_capacity'))"
  for N in 9 10; do
    env $e timeout -k 10 200 python -u bench.py --cpu-baseline 0 --config4-steps 0 --rm-count $N --steps 5 --warmup 1 --no-hint-steps 5 > $O/b${N}_${e#*=}.json 2> $O/b${N}_${e#*=}.err || { tail -5 $O/b${N}_${e#*=}.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/b${N}_${e#*=}.json').read().strip().splitlines()[-1]); n=d['no_hint']; print('2pc$N [$e] hinted', round(d['ms_per_step'],4), 'no_hint', round(n['ms_per_step'],4), 'vs', round(n['vs_value'],3), 'rehashes', n.get('rehashes'), 'cap', n.get('table_capacity'))"
  done
done
echo "growstep ok"
