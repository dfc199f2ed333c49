#!/bin/bash
# Round 6: probe rounds (SR_PROBE_BATCH=1) against per-lane queues (-4) at the new table sizes
# (2pc N=9: 2^26 4-byte slots; N=10: 2^28; N=11: 2^31).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_env_ab.sh r06pl9 2 "SR_PROBE_BATCH=1" "SR_PROBE_BATCH=-4" -- --steps 20 || exit 1
bash scripts/gpu_env_ab.sh r06pl10 2 "SR_PROBE_BATCH=1" "SR_PROBE_BATCH=-4" -- --rm-count 10 --steps 5 --warmup 1 || exit 1
bash scripts/gpu_env_ab.sh r06pl11 1 "SR_PROBE_BATCH=1" "SR_PROBE_BATCH=-4" -- --rm-count 11 --steps 2 --warmup 1 || exit 1
echo "probeloop ok"
