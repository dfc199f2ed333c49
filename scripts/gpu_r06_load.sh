#!/bin/bash
# Round 6: the visited set's planned load at the capacity hint (SR_TABLE_LOAD, default 0.5) with 32-bit
# slots: 2pc N=9 (2^25 vs 2^26 slots), N=10, N=11.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_env_ab.sh r06load9 3 "SR_TABLE_LOAD=0.5" "SR_TABLE_LOAD=0.3" "SR_TABLE_LOAD=0.2" -- --steps 20 || exit 1
bash scripts/gpu_env_ab.sh r06load10 2 "SR_TABLE_LOAD=0.5" "SR_TABLE_LOAD=0.3" -- --rm-count 10 --steps 5 --warmup 1 || exit 1
bash scripts/gpu_env_ab.sh r06load11 1 "SR_TABLE_LOAD=0.5" "SR_TABLE_LOAD=0.3" -- --rm-count 11 --steps 2 --warmup 1 || exit 1
echo "load ok"
