#!/bin/bash
# Round 6: the asynchronous early growth (no capacity hint): whole GPU suite, then 2pc N=9 and
# increment_lock N=11 without a hint, early growth on and off.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r06nh2}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "growth or hint or doubl or grow or parity" > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
SR_VERBOSE_NOHINT=1 timeout -k 10 120 python -u scripts/nohint_verbose.py > $O/verbose.txt 2>&1 || { tail -20 $O/verbose.txt; exit 1; }
for r in 1 2 3; do
  for e in "SR_EARLY_GROW_MAX=131072" "SR_EARLY_GROW_MAX=0"; do
    env $e timeout -k 10 200 python -u bench.py --cpu-baseline 0 --config4-steps 0 --steps 20 --no-hint-steps 20 > $O/b9_${e#*=}_$r.json 2> $O/b9_${e#*=}_$r.err || { tail -5 $O/b9_${e#*=}_$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/b9_${e#*=}_$r.json').read().strip().splitlines()[-1]); n=d['no_hint']; print('2pc9 [$e] r$r hinted', round(d['ms_per_step'],4), 'no_hint', round(n['ms_per_step'],4), 'vs', round(n['vs_value'],3), 'rehashes', n.get('rehashes'))"
  done
done
echo "nohint2 ok"
