#!/bin/bash
# Round 6: the arena's growth step of unhinted checks (default 8 against SR_ARENA_STEP = 4; a first run compared 4 / 8 / 16), no_hint ms.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06as
mkdir -p "$O"
for r in 1 2; do
  for e in "SR_X=0" "SR_ARENA_STEP=4"; do
    for args in "--rm-count 9 --no-hint-steps 10" "--rm-count 10 --no-hint-steps 4" "--model increment_lock --threads 11 --no-hint-steps 2"; do
      tag=$(echo "$args" | tr -d ' -' | cut -c1-12)
      env $e timeout -k 10 200 python -u bench.py --cpu-baseline 0 --config4-steps 0 --steps 1 --warmup 1 $args \
          > "$O/${tag}_${e}_$r.json" 2> "$O/${tag}_${e}_$r.err" || { tail -5 "$O/${tag}_${e}_$r.err"; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/${tag}_${e}_$r.json').read().strip().splitlines()[-1]); n=d['no_hint']; print('$e r$r $args', 'hinted', round(d['ms_per_step'],3), 'no_hint', round(n['ms_per_step'],3))"
    done
  done
done
echo "arena step ok"
