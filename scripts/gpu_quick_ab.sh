#!/bin/bash
# Waves per workgroup of expand_fast for narrow states (SR_NARROW_WPB: the LDS duplicate filter's reach is
# the workgroup's chunk of waves x ppw parents) x the filter size (SR_FILTER_LOG2), 2pc N=9: ms per check
# and visited-set probes per check (counting pass). cur = WPB 4.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-q}
O=gpurun_out/$T
mkdir -p $O
export SR_LIB_DIGEST_CHECK=0
LIB=stateright_amd/libstateright_gpu.so
cp "$LIB" gpurun_ab/lib_cur.so || exit 1
for v in wpb8 wpb16; do
    cp gpurun_ab/lib_$v.so "$LIB" || exit 1
    timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "two_phase or 2pc or tp or config" --timeout 120 --timeout-method thread > $O/parity_$v.log 2>&1 || { tail -30 $O/parity_$v.log; cp gpurun_ab/lib_cur.so "$LIB"; exit 1; }
    echo "$v $(tail -1 $O/parity_$v.log)"
done
run() {  # label lib env -- bench args
    local label=$1 lib=$2; shift 2
    local envs=()
    while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
    cp "gpurun_ab/lib_$lib.so" "$LIB" || exit 1
    env "${envs[@]}" timeout -k 10 200 python -u bench.py --cpu-baseline 0 --config4-steps 0 --no-hint-steps 0 "$@" > "$O/$label.json" 2> "$O/$label.err" || { tail -5 "$O/$label.err"; cp gpurun_ab/lib_cur.so "$LIB"; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/$label.json').read().strip().splitlines()[-1]); l=d.get('levels') or {}; r=d['roofline']; print('$label', round(d['ms_per_step'],4), 'small', round(l.get('small_levels_ms',0),4), 'big', round(l.get('big_levels_ms',0),4), 'probes', round(r.get('probes_per_step',0)/1e6,2), 'M')"
}
for r in 1 2; do
    run cur_f9_r$r cur SR_FILTER_LOG2=9 -- --steps 50 --warmup 3 || exit 1
    run wpb8_f9_r$r wpb8 SR_FILTER_LOG2=9 -- --steps 50 --warmup 3 || exit 1
    run wpb8_f10_r$r wpb8 SR_FILTER_LOG2=10 -- --steps 50 --warmup 3 || exit 1
    run wpb8_f11_r$r wpb8 SR_FILTER_LOG2=11 -- --steps 50 --warmup 3 || exit 1
    run wpb16_f11_r$r wpb16 SR_FILTER_LOG2=11 -- --steps 50 --warmup 3 || exit 1
    run wpb16_f12_r$r wpb16 SR_FILTER_LOG2=12 -- --steps 50 --warmup 3 || exit 1
done
cp gpurun_ab/lib_cur.so "$LIB"
echo "quick ab ok"
