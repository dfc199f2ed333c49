#!/bin/bash
# Direct-exchange state kept across checks: parity tests, then the one-rank RCCL check time with the
# direct exchange and with RCCL's all-to-all, and 2pc N=9 over virtual partitions / in-process ranks.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03r
mkdir -p $O
timeout -k 10 60 ./scripts/ipc_selftest > $O/ipc.log 2>&1 || { cat $O/ipc.log; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_partitioned.py tests/test_gpu_dist_ranks.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for d in 1 0; do
  SR_DIRECT=$d timeout -k 10 300 python -u bench.py --mode rccl1 --steps 20 --warmup 3 --cpu-baseline 0 --config4-steps 0 > $O/rccl1_direct$d.json 2> $O/rccl1_direct$d.err || { tail -5 $O/rccl1_direct$d.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/rccl1_direct$d.json')); print('rccl1 direct=$d', round(d['ms_per_step'],3), 'ms', d['config']['parallelism'])"
done
GPU_MAX_HW_QUEUES=16 REPS=5 timeout -k 10 300 python -u scripts/time_partitioned.py 9 > $O/time9.log 2>&1 || { tail $O/time9.log; exit 1; }
grep -v "version\|Hostname\|path" $O/time9.log
SR_HEAD_MAX=0 GPU_MAX_HW_QUEUES=16 REPS=5 timeout -k 10 300 python -u scripts/time_partitioned.py 9 > $O/time9_nohead.log 2>&1 || { tail $O/time9_nohead.log; exit 1; }
echo "== SR_HEAD_MAX=0"; grep -v "version\|Hostname\|path" $O/time9_nohead.log
