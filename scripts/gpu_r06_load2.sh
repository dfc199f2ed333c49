#!/bin/bash
# Round 6: lower planned loads (SR_TABLE_LOAD 0.3 against 0.12-0.15), the first no-hint growth step
# (SR_GROW_FIRST), and the partition tables' planned load (SR_PART_LOAD) for config 4.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06load2
mkdir -p $O
bash scripts/gpu_env_ab.sh r06load9b 2 "SR_TABLE_LOAD=0.3" "SR_TABLE_LOAD=0.12" -- --steps 20 || exit 1
bash scripts/gpu_env_ab.sh r06load10b 1 "SR_TABLE_LOAD=0.3" "SR_TABLE_LOAD=0.15" -- --rm-count 10 --steps 5 --warmup 1 || exit 1
bash scripts/gpu_env_ab.sh r06load11b 1 "SR_TABLE_LOAD=0.3" "SR_TABLE_LOAD=0.15" -- --rm-count 11 --steps 2 --warmup 1 || exit 1
bash scripts/gpu_env_ab.sh r06loadil 1 "SR_TABLE_LOAD=0.5" "SR_TABLE_LOAD=0.3" -- --model increment_lock --threads 11 --steps 2 --warmup 1 || exit 1
for e in "SR_GROW_FIRST=0" "SR_GROW_FIRST=16"; do
  for N in 9 10; do
    env $e timeout -k 10 200 python -u bench.py --cpu-baseline 0 --config4-steps 0 --rm-count $N --steps 5 --warmup 1 --no-hint-steps 5 > $O/b${N}_${e#*=}.json 2> $O/b${N}_${e#*=}.err || { tail -5 $O/b${N}_${e#*=}.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/b${N}_${e#*=}.json').read().strip().splitlines()[-1]); n=d['no_hint']; print('2pc$N [$e] hinted', round(d['ms_per_step'],4), 'no_hint', round(n['ms_per_step'],4), 'vs', round(n['vs_value'],3), 'rehashes', n.get('rehashes'), 'cap', n.get('table_capacity'))"
  done
  env $e timeout -k 10 300 python -u bench.py --cpu-baseline 0 --config4-steps 0 --model increment_lock --threads 11 --steps 2 --warmup 1 --no-hint-steps 3 > $O/il11_${e#*=}.json 2> $O/il11_${e#*=}.err || { tail -5 $O/il11_${e#*=}.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/il11_${e#*=}.json').read().strip().splitlines()[-1]); n=d['no_hint']; print('inclock11 [$e] hinted', round(d['ms_per_step'],3), 'no_hint', round(n['ms_per_step'],3), 'vs', round(n['vs_value'],3), 'rehashes', n.get('rehashes'), 'cap', n.get('table_capacity'))"
done
for T in 8 4; do bash scripts/gpu_okey_sweep.sh 11 $T "SR_PART_LOAD=0.5" "SR_PART_LOAD=0.3" || exit 1; done
echo "load2 ok"
