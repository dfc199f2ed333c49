#!/bin/bash
# Round 6: the arena step on unhinted paxos C=6 (default 8 against SR_ARENA_STEP = 4), no_hint ms.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06asp
mkdir -p "$O"
for r in 1 2 3; do
  for e in "SR_X=0" "SR_ARENA_STEP=4"; do
    env $e timeout -k 10 200 python -u bench.py --cpu-baseline 0 --config4-steps 0 --steps 3 --warmup 1 --model paxos --clients 6 --no-hint-steps 5 \
        > "$O/${e}_$r.json" 2> "$O/${e}_$r.err" || { tail -5 "$O/${e}_$r.err"; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/${e}_$r.json').read().strip().splitlines()[-1]); n=d['no_hint']; print('$e r$r', 'hinted', round(d['ms_per_step'],3), 'no_hint', round(n['ms_per_step'],3), n['rehashes'], n['table_capacity'])"
  done
done
echo "arena step paxos ok"
