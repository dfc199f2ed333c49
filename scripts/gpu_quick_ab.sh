#!/bin/bash
# Non-temporal frontier stores (lib_nt: -DSR_NT_FRONTIER) against the current library, 2pc N=9: ms per check
# and a kernel trace of each (the idle time before big levels).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-q}
O=gpurun_out/$T
mkdir -p $O
export SR_LIB_DIGEST_CHECK=0
LIB=stateright_amd/libstateright_gpu.so
cp "$LIB" gpurun_ab/lib_cur.so || exit 1
run() {  # label lib -- bench args
    local label=$1 lib=$2; shift 3
    cp "gpurun_ab/lib_$lib.so" "$LIB" || exit 1
    timeout -k 10 200 python -u bench.py --cpu-baseline 0 --config4-steps 0 --no-hint-steps 0 "$@" > "$O/$label.json" 2> "$O/$label.err" || { tail -5 "$O/$label.err"; cp gpurun_ab/lib_cur.so "$LIB"; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/$label.json').read().strip().splitlines()[-1]); l=d.get('levels') or {}; print('$label', round(d['ms_per_step'],4), 'small', round(l.get('small_levels_ms',0),4), 'big', round(l.get('big_levels_ms',0),4))"
}
for r in 1 2 3; do
    run tp9_cur_r$r cur -- --steps 50 --warmup 3 || exit 1
    run tp9_nt_r$r nt -- --steps 50 --warmup 3 || exit 1
done
cp gpurun_ab/lib_nt.so "$LIB"
bash scripts/ktrace.sh $T/kt_nt --steps 20 --warmup 3 --cpu-baseline 0 --config4-steps 0 --no-hint-steps 0 || { cp gpurun_ab/lib_cur.so "$LIB"; exit 1; }
cp gpurun_ab/lib_cur.so "$LIB"
echo "quick ab ok"
