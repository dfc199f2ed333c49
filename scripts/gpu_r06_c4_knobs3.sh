#!/bin/bash
# Round 6: the smaller route stages at T = 2 and 4 (config 4 on 2 and 4 virtual partitions).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
for T in 2 4; do
bash scripts/gpu_okey_sweep.sh 11 $T "SR_X=0" "SR_RSTAGE_WORDS=512 SR_LSTAGE_WORDS=512" || exit 1
done
echo "c4 knobs3 ok"
