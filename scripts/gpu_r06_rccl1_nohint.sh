#!/bin/bash
# Round 6: where the partitioned path's unhinted check (2pc N=9, one RCCL rank) loses to the hinted one:
# a kernel trace of 3 hinted + 3 unhinted checks.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/ktrace.sh r06rccl1 --mode rccl1 --steps 3 --warmup 1 --no-hint-steps 3 --cpu-baseline 0 --config4-steps 0 || exit 1
echo "rccl1 trace ok"
