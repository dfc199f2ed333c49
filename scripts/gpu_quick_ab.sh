#!/bin/bash
# The owner-ordered record flush (RF_ORDERED) forced on one device: the partitioned, in-process-rank
# and process-rank parity tests under it, then config 4 on 8 virtual partitions both ways.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-q}
O=gpurun_out/$T
mkdir -p $O
SR_ORDERED_FLUSH=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_partitioned.py tests/test_gpu_dist_ranks.py tests/test_gpu_shm_ranks.py tests/test_gpu_visitors.py tests/test_gpu_eventually.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/parity_ordered.log 2>&1 || { tail -30 $O/parity_ordered.log; exit 1; }
tail -1 $O/parity_ordered.log
bash scripts/gpu_okey_sweep.sh 11 8 "SR_ORDERED_FLUSH=0" "SR_ORDERED_FLUSH=1" || exit 1
