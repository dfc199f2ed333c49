#!/bin/bash
# Config 4 (2pc N=11) on 8 virtual partitions: the route kernel's probe loops (kernel traces and the
# per-partition critical path, scripts/gpu_okey_sweep.sh), after a parity check of the queue form.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-q}
O=gpurun_out/$T
mkdir -p $O
SR_ROUTE_QUEUE=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_partitioned.py tests/test_gpu_dist_ranks.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/parity_rq.log 2>&1 || { tail -30 $O/parity_rq.log; exit 1; }
tail -1 $O/parity_rq.log
bash scripts/gpu_okey_sweep.sh 11 8 "SR_ROUTE_QUEUE=0" "SR_ROUTE_QUEUE=1" || exit 1
