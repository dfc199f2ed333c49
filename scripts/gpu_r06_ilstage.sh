#!/bin/bash
# Round 6: narrow stages in states (increment_lock's two-word states get twice the stage): the
# increment / increment_lock GPU tests, then the grid residencies again at the new stage.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06ils
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "increment or lock or growth or rehash or doubling or probe" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash scripts/gpu_env_ab.sh r06ils/il11 2 "SR_X=0" "SR_GRID_RES=2" "SR_GRID_RES=8" -- --steps 2 --warmup 1 --model increment_lock --threads 11 || exit 1
bash scripts/gpu_env_ab.sh r06ils/il10 2 "SR_X=0" "SR_GRID_RES=2" "SR_GRID_RES=8" -- --steps 5 --warmup 1 --model increment_lock --threads 10 || exit 1
echo "ilstage ok"
