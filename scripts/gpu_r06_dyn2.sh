#!/bin/bash
# Round 6: dynamic chunks as a separate kernel instantiation for deep levels (> DYN_MIN_RATIO chunks per
# workgroup, chosen by the host) against none (SR_DYN=0): the whole GPU suite, then every deep config.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06dyn2
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash scripts/gpu_env_ab.sh r06dyn2/n9 3 "SR_DYN=0" "SR_X=0" -- --steps 20 || exit 1
bash scripts/gpu_env_ab.sh r06dyn2/n10 2 "SR_DYN=0" "SR_X=0" -- --steps 5 --rm-count 10 || exit 1
bash scripts/gpu_env_ab.sh r06dyn2/n11 2 "SR_DYN=0" "SR_X=0" -- --steps 2 --warmup 1 --rm-count 11 || exit 1
bash scripts/gpu_env_ab.sh r06dyn2/il11 2 "SR_DYN=0" "SR_X=0" -- --steps 2 --warmup 1 --model increment_lock --threads 11 || exit 1
bash scripts/gpu_env_ab.sh r06dyn2/il10 2 "SR_DYN=0" "SR_X=0" -- --steps 5 --warmup 1 --model increment_lock --threads 10 || exit 1
echo "dyn2 ok"
