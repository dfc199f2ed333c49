#!/bin/bash
# Paxos expand A/B: the in-tree engine against build_ab/lib_<v>.so (paxos C=3 bench lines), after
# the paxos parity tests through the new build.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/paxos_ab
mkdir -p "$O"
SR_LIB_PATH=build_ab/lib_s3584.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "paxos" --timeout 120 --timeout-method thread > "$O/parity.log" 2>&1 || { tail -30 "$O/parity.log"; exit 1; }
tail -1 "$O/parity.log"
for rep in 1 2 3; do
for v in head s2048 s3584; do
    lib=build_ab/lib_$v.so; [ $v = head ] && lib=stateright_amd/libstateright_gpu.so
    SR_LIB_PATH=$lib timeout -k 10 120 python -u bench.py --model paxos --steps 20 --warmup 3 --cpu-baseline 0 --config4-steps 0 > "$O/p_$v.json" 2> "$O/p_$v.err" || { tail -20 "$O/p_$v.err"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('paxos', sys.argv[2], round(d['ms_per_step'],3), 'kernel_us_peak', max(d['levels']['kernel_us']), 'sum', round(sum(d['levels']['kernel_us']),1))" "$O/p_$v.json" $v
done
done
