#!/bin/bash
# Round 6: the owner key's width (RMs) with the multiplicative owner hash, T = 8 / 4 / 2.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
for T in 8 4 2; do bash scripts/gpu_okey_sweep.sh 11 $T "SR_OWNER_RMS=4" "SR_OWNER_RMS=3" "SR_OWNER_RMS=5" || exit 1; done
echo "okey rms ok"
