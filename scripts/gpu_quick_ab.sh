#!/bin/bash
# Small levels: parents per wave down to 1 (SR_PPW_MIN_LOG2) with the map-free one-parent path.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-q}
O=gpurun_out/$T
mkdir -p $O
SR_PPW_MIN_LOG2=0 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_eventually.py tests/test_gpu_symmetry.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
bash scripts/gpu_env_ab.sh $T/ab9 3 "" "SR_PPW_MIN_LOG2=1" "SR_PPW_MIN_LOG2=0" "SR_PPW_MIN_LOG2=0 SR_PPW_WAVES=2048" -- --steps 20 --warmup 3 || exit 1
