#!/bin/bash
# Round 6: config 4 (2pc N=11, 8 virtual partitions) under route-kernel knobs: parents per wave,
# record / local stage sizes (LDS per block), the duplicate filter, the owner key's width.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_okey_sweep.sh 11 8 "SR_X=0" "SR_ROUTE_PPW_LOG2=5" "SR_ROUTE_PPW_LOG2=4" "SR_RSTAGE_WORDS=512" "SR_LSTAGE_WORDS=512" "SR_RSTAGE_WORDS=512 SR_LSTAGE_WORDS=512" "SR_FILTER_LOG2=0" "SR_OWNER_RMS=3" "SR_OWNER_RMS=5" || exit 1
echo "c4 knobs ok"
