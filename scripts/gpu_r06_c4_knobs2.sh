#!/bin/bash
# Round 6: config 4's route kernel LDS (record stage, local stage, filter) around the smaller stages.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_okey_sweep.sh 11 8 "SR_RSTAGE_WORDS=512 SR_LSTAGE_WORDS=512" "SR_RSTAGE_WORDS=256 SR_LSTAGE_WORDS=512" "SR_RSTAGE_WORDS=512 SR_LSTAGE_WORDS=256" "SR_RSTAGE_WORDS=256 SR_LSTAGE_WORDS=256" "SR_RSTAGE_WORDS=512 SR_LSTAGE_WORDS=512 SR_FILTER_LOG2=8" "SR_RSTAGE_WORDS=384 SR_LSTAGE_WORDS=384" "SR_RSTAGE_WORDS=512 SR_LSTAGE_WORDS=512 SR_ROUTE_GRID_MAX=4096" || exit 1
echo "c4 knobs2 ok"
