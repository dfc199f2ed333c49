#!/bin/bash
# Config 4 (2pc N=11) on 8 virtual partitions: the insert kernel's probe form (kernel traces and the
# per-partition critical path, scripts/gpu_okey_sweep.sh), after the partitioned parity tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-q}
O=gpurun_out/$T
mkdir -p $O
SR_INSERT_BATCH_MIN=1000 timeout -k 10 600 python -u -m pytest tests/test_gpu_partitioned.py tests/test_gpu_dist_ranks.py tests/test_gpu_shm_ranks.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
bash scripts/gpu_okey_sweep.sh 11 8 "SR_INSERT_MACHINES=0" "SR_INSERT_MACHINES=1" || exit 1
