#!/bin/bash
# The whole -m gpu suite, then a same-box A/B of the round-4 library against the current one.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-q}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
bash scripts/gpu_lib_ab.sh $T/lib9 3 -- --steps 20 --warmup 3 || exit 1
bash scripts/gpu_env_ab.sh $T/rccl1 2 "" -- --mode rccl1 --steps 10 --warmup 3
