#!/bin/bash
# One-rank RCCL communicator, 2pc N=9: direct exchange vs RCCL all-to-all, alternating, 3 runs each.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/rccl1_ab
mkdir -p $O
for k in 1 2 3; do
  for d in 1 0; do
    SR_DIRECT=$d timeout -k 10 300 python -u bench.py --mode rccl1 --steps 30 --warmup 5 --cpu-baseline 0 --config4-steps 0 > $O/d${d}_$k.json 2> $O/d${d}_$k.err || { tail -5 $O/d${d}_$k.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/d${d}_$k.json')); print('direct=$d run $k', round(d['ms_per_step'],3), 'ms')"
  done
done
