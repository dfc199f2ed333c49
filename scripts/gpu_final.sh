#!/bin/bash
# End-of-round measurements on one MI355X at the committed sources, every GPU step under its own
# time limit and stopping at the first failure:
#   scripts/gpu_final.sh <tag>
# 1. the whole -m gpu suite; 2. the default bench line and the side configurations (scripts/
# gpu_round.sh); 3. rocprofv3 kernel stats; 4. the PMC request ceilings and per-config traffic
# stamped with the source digest (scripts/gpu_roofline.sh); 5. the multi-process rehearsal of
# bench.py --gpus 2 on this one GPU (shared-memory host transport).
set -o pipefail
TAG=${1:?tag}
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_round.sh $TAG tests || exit 1
bash scripts/gpu_round.sh $TAG bench || exit 1
bash scripts/gpu_round.sh $TAG prof || exit 1
bash scripts/gpu_roofline.sh || exit 1
timeout -k 10 400 python -u bench.py --gpus 2 --comm shm --steps 5 --warmup 2 --config4-steps 1 > gpurun_out/$TAG/shm_n2.json 2> gpurun_out/$TAG/shm_n2.err || { tail -5 gpurun_out/$TAG/shm_n2.err; exit 1; }
echo "final ok"
