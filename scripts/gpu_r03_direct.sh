#!/bin/bash
# Direct exchange checks on one MI355X: the cross-process IPC self-test, the partitioned and
# in-process-rank parity tests, 2pc N=9 over T virtual partitions / in-process ranks, and the route
# and insert kernel time of 2pc N=11 at T = 8 under the defaults.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03q
mkdir -p $O
timeout -k 10 60 ./scripts/ipc_selftest > $O/ipc.log 2>&1; rc=$?; cat $O/ipc.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_partitioned.py tests/test_gpu_dist_ranks.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
GPU_MAX_HW_QUEUES=16 REPS=5 timeout -k 10 300 python -u scripts/time_partitioned.py 9 > $O/time9.log 2>&1 || { tail $O/time9.log; exit 1; }
cat $O/time9.log
bash scripts/gpu_route_knobs.sh 11 8 "" || exit 1
