#!/bin/bash
# enabled_slot models (paxos, ...): the successor map written straight from the enabled pass's ballots
# (current) against the per-parent walk (lib_old); actor/paxos parity first, then ms per check, alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-q}
O=gpurun_out/$T
mkdir -p $O
export SR_LIB_DIGEST_CHECK=0
LIB=stateright_amd/libstateright_gpu.so
cp "$LIB" gpurun_ab/lib_cur.so || exit 1
timeout -k 10 500 python -u -m pytest tests/test_gpu_actor.py tests/test_gpu_parity.py tests/test_gpu_fingerprints.py -m gpu -x -q -k "paxos or actor or single or abd or ping or register or fingerprint" --timeout 120 --timeout-method thread > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
run() {  # label lib -- bench args
    local label=$1 lib=$2; shift 3
    cp "gpurun_ab/lib_$lib.so" "$LIB" || exit 1
    timeout -k 10 200 python -u bench.py --cpu-baseline 0 --config4-steps 0 --no-hint-steps 0 "$@" > "$O/$label.json" 2> "$O/$label.err" || { tail -5 "$O/$label.err"; cp gpurun_ab/lib_cur.so "$LIB"; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/$label.json').read().strip().splitlines()[-1]); l=d.get('levels') or {}; print('$label', round(d['ms_per_step'],4), 'small', round(l.get('small_levels_ms',0),4), 'big', round(l.get('big_levels_ms',0),4))"
}
for r in 1 2 3; do
    for v in old cur; do
        run px3_${v}_r$r $v -- --model paxos --clients 3 --steps 200 --warmup 5 || exit 1
        run px6_${v}_r$r $v -- --model paxos --clients 6 --steps 30 --warmup 2 || exit 1
    done
done
cp gpurun_ab/lib_cur.so "$LIB"
echo "quick ab ok"
