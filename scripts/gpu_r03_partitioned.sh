#!/bin/bash
# Round-3 partitioned-search measurements on one MI355X (run through gpurun from the repo root):
# the partitioned / in-process-rank parity tests, then route/insert kernel time per check for 2pc
# N=11 over T virtual partitions under the self-record and exchange knobs, then the one-rank RCCL
# communicator's check time with the direct exchange and with RCCL's all-to-all.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03p
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_partitioned.py tests/test_gpu_dist_ranks.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash scripts/gpu_route_knobs.sh 11 8 "" "SR_SELF_RECORDS_MIN=0" "SR_RSTAGE_WORDS=2048" || exit 1
bash scripts/gpu_route_knobs.sh 11 4 "" "SR_SELF_RECORDS_MIN=0" || exit 1
bash scripts/gpu_route_knobs.sh 11 2 "SR_SELF_RECORDS_MIN=2" "SR_SELF_RECORDS_MIN=0" || exit 1
for d in 1 0; do
  SR_DIRECT=$d timeout -k 10 300 python -u bench.py --mode rccl1 --steps 20 --warmup 3 --cpu-baseline 0 --config4-steps 0 > $O/rccl1_direct$d.json 2> $O/rccl1_direct$d.err || { tail -5 $O/rccl1_direct$d.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/rccl1_direct$d.json')); print('rccl1 direct=$d', round(d['ms_per_step'],3), 'ms', d['config']['parallelism'])"
done
