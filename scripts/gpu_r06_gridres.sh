#!/bin/bash
# Round 6: one residency per expand grid (the new default) against two (SR_GRID_RES=2): the whole
# GPU suite on the new default, then every bench workload alternately.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06gr
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash scripts/gpu_env_ab.sh r06gr/n9 3 "SR_GRID_RES=2" "SR_X=0" -- --steps 20 || exit 1
bash scripts/gpu_env_ab.sh r06gr/p3 3 "SR_GRID_RES=2" "SR_X=0" -- --steps 20 --model paxos --clients 3 || exit 1
bash scripts/gpu_env_ab.sh r06gr/p6 2 "SR_GRID_RES=2" "SR_X=0" -- --steps 5 --model paxos --clients 6 || exit 1
bash scripts/gpu_env_ab.sh r06gr/sc4 2 "SR_GRID_RES=2" "SR_X=0" -- --steps 10 --model single_copy --clients 4 || exit 1
bash scripts/gpu_env_ab.sh r06gr/il11 1 "SR_GRID_RES=2" "SR_X=0" -- --steps 2 --warmup 1 --model increment_lock --threads 11 || exit 1
bash scripts/gpu_env_ab.sh r06gr/n10 2 "SR_GRID_RES=2" "SR_X=0" -- --steps 5 --rm-count 10 || exit 1
echo "gridres ok"
