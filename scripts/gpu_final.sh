#!/bin/bash
# Last GPU pass at the current sources: the whole -m gpu suite, the no-hint growth log of 2pc N=9, the
# default bench line and the side configurations, the rocprofv3 kernel stats, then the PMC traffic and
# ceilings stamped with the source digest (scripts/gpu_roofline.sh). Stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-final}
bash scripts/gpu_round.sh $T tests || exit 1
timeout -k 10 200 python -u scripts/nohint_verbose.py > gpurun_out/$T/nohint_verbose.log 2>&1 || exit 1
bash scripts/gpu_round.sh $T bench || exit 1
bash scripts/gpu_round.sh $T prof || exit 1
bash scripts/gpu_roofline.sh || exit 1
echo "final pass ok"
