#!/bin/bash
# Round 6: per-lane probe queues for claim-heavy levels (SR_QUEUE_RATIO) on 2pc N=9 and N=10.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_env_ab.sh r06qr 2 "SR_QUEUE_RATIO=0" "SR_QUEUE_RATIO=1.2" "SR_QUEUE_RATIO=1.6" "SR_QUEUE_RATIO=2.2" -- --steps 20 || exit 1
for f in gpurun_out/r06qr/e*_r2.json; do echo $f; python3 scripts/level_attribution.py $f | tail -2; done
echo "queue ratio ok"
