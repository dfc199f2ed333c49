#!/bin/bash
# Round 6: growth by ranges (rehash_ranges) against the CAS rehash, SR_REHASH_RANGES = 1 / 0: the
# growth tests, then unhinted checks (bench.py's no_hint line) of 2pc N=9 / N=10 and increment_lock N=11.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06rh
mkdir -p "$O"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread \
    -k "rehash or grow" > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
tail -3 "$O/tests.log"
for r in 1; do
  for e in 1 0; do
    for args in "--rm-count 9 --no-hint-steps 10" "--rm-count 10 --no-hint-steps 3" "--model increment_lock --threads 11 --no-hint-steps 2"; do
      tag=$(echo "$args" | tr -d ' -' | cut -c1-24)
      SR_REHASH_RANGES=$e timeout -k 10 200 python -u bench.py --cpu-baseline 0 --config4-steps 0 --steps 2 --warmup 1 $args \
          > "$O/${tag}_e${e}_r$r.json" 2> "$O/${tag}_e${e}_r$r.err" || { tail -5 "$O/${tag}_e${e}_r$r.err"; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/${tag}_e${e}_r$r.json').read().strip().splitlines()[-1]); n=d['no_hint']; print('ranges=$e r$r $args', 'hinted', round(d['ms_per_step'],3), 'no_hint', round(n['ms_per_step'],3), round(n['vs_value'],3))"
    done
  done
done
echo "rehash ab ok"
