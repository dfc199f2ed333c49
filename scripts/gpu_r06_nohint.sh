#!/bin/bash
# Round 6: checks without capacity_hint (the reference user's path), early growth on (default) and
# off (SR_EARLY_GROW_MAX=0): 2pc N=9 and increment_lock N=11, hinted value beside.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r06nh}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "growth or hint or doubl or grow" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for e in "SR_EARLY_GROW_MAX=131072" "SR_EARLY_GROW_MAX=0"; do
    env $e timeout -k 10 200 python -u bench.py --cpu-baseline 0 --config4-steps 0 --steps 20 --no-hint-steps 20 > $O/b9_${e#*=}_$r.json 2> $O/b9_${e#*=}_$r.err || { tail -5 $O/b9_${e#*=}_$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/b9_${e#*=}_$r.json').read().strip().splitlines()[-1]); n=d['no_hint']; print('2pc9 [$e] r$r hinted', round(d['ms_per_step'],4), 'no_hint', round(n['ms_per_step'],4), 'vs', round(n['vs_value'],3), 'rehashes', n.get('rehashes'))"
    env $e timeout -k 10 300 python -u bench.py --cpu-baseline 0 --config4-steps 0 --model increment_lock --threads 11 --steps 3 --warmup 1 --no-hint-steps 3 > $O/il11_${e#*=}_$r.json 2> $O/il11_${e#*=}_$r.err || { tail -5 $O/il11_${e#*=}_$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/il11_${e#*=}_$r.json').read().strip().splitlines()[-1]); n=d['no_hint']; print('inclock11 [$e] r$r hinted', round(d['ms_per_step'],3), 'no_hint', round(n['ms_per_step'],3), 'vs', round(n['vs_value'],3), 'rehashes', n.get('rehashes'))"
  done
done

# config 4 on 8 virtual partitions with 32-bit quotient slots (default) and 8-byte ones
bash scripts/gpu_okey_sweep.sh 11 8 "SR_SLOT32=1" "SR_SLOT32=0" > $O/config4.txt 2>&1 || { tail -20 $O/config4.txt; exit 1; }
cat $O/config4.txt
echo "nohint ok"
