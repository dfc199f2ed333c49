#!/bin/bash
# Round 6: unhinted partitioned checks growing to the planned load (dist.hpp grow_at): GPU suite,
# then the partitioned lines (one RCCL rank; two processes on one GPU) with their no_hint fields.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06pn
mkdir -p "$O"
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/gpu_tests.log" 2>&1 || { tail -40 "$O/gpu_tests.log"; exit 1; }
tail -2 "$O/gpu_tests.log"
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --mode rccl1 --steps 10 --warmup 3 --cpu-baseline 0 --config4-steps 0 > "$O/rccl1_$r.json" 2> "$O/rccl1_$r.err" || { tail -5 "$O/rccl1_$r.err"; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/rccl1_$r.json').read().strip().splitlines()[-1]); n=d['no_hint']; print('rccl1', round(d['ms_per_step'],3), 'no_hint', round(n['ms_per_step'],3), round(n['vs_value'],3), 'rehashes', n['rehashes'], 'cap', n['table_capacity'])"
done
timeout -k 10 300 python -u bench.py --gpus 2 --comm shm --steps 10 --warmup 2 --config4-steps 1 > "$O/shm2.json" 2> "$O/shm2.err" || { tail -20 "$O/shm2.err"; exit 1; }
python3 -c "import json; d=json.loads(open('$O/shm2.json').read().strip().splitlines()[-1]); n=d['no_hint']; print('shm2', round(d['ms_per_step'],3), 'no_hint', round(n['ms_per_step'],3), round(n['vs_value'],3), 'config4', d['config4']['ms_per_step'])"
echo "partitioned no-hint ok"
