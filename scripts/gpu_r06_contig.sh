#!/bin/bash
# Round 6: the visited set in physically contiguous device memory (SR_TABLE_KIND=3,
# hipDeviceMallocContiguous: larger translation fragments) against ordinary hipMalloc memory,
# 2pc N=11 / 10 / 9 alternately.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_env_ab.sh r06contig/n11 2 "SR_X=0" "SR_TABLE_KIND=3" -- --steps 2 --warmup 1 --rm-count 11 || exit 1
bash scripts/gpu_env_ab.sh r06contig/n10 2 "SR_X=0" "SR_TABLE_KIND=3" -- --steps 5 --rm-count 10 || exit 1
bash scripts/gpu_env_ab.sh r06contig/n9 2 "SR_X=0" "SR_TABLE_KIND=3" -- --steps 20 || exit 1
echo "contig ok"
