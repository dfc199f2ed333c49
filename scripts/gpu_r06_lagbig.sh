#!/bin/bash
# Round 6: the partitioned pipelined loop's "big level" rule (a level whose planned frontier passes
# SR_LAG_BIG, default 262144, is enqueued only after the previous level's rows are read: one host
# round trip per big level) against never waiting (SR_LAG_BIG=1e12): the one-rank RCCL path and two
# processes on one GPU, 2pc N=9.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_env_ab.sh r06lag/rccl1 3 "SR_X=0" "SR_LAG_BIG=1000000000000" -- --mode rccl1 --steps 10 || exit 1
bash scripts/gpu_env_ab.sh r06lag/shm2 2 "SR_X=0" "SR_LAG_BIG=1000000000000" -- --gpus 2 --comm shm --steps 10 || exit 1
echo "lagbig ok"
