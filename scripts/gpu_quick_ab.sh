#!/bin/bash
# No capacity hint, 2pc N=9 / N=10 / paxos C=6: the arena grown with the visited set (current) against the
# previous library (lib_old: the arena's own step a level later), alternating; 20 no-hint checks per run.
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
    timeout -k 10 200 python -u bench.py --cpu-baseline 0 --config4-steps 0 "$@" > "$O/$label.json" 2> "$O/$label.err" || { tail -5 "$O/$label.err"; cp gpurun_ab/lib_cur.so "$LIB"; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/$label.json').read().strip().splitlines()[-1]); nh=d.get('no_hint') or {}; print('$label', round(d['ms_per_step'],4), 'nohint', round(nh.get('ms_per_step',0),4), nh.get('table_capacity'), nh.get('rehashes'))"
}
for r in 1 2 3; do
    for v in old cur; do
        run tp9_${v}_r$r $v -- --steps 10 --warmup 2 --no-hint-steps 20 || exit 1
    done
done
for v in old cur; do
    run tp10_${v} $v -- --rm-count 10 --steps 3 --warmup 1 --no-hint-steps 5 || exit 1
    run px6_${v} $v -- --model paxos --clients 6 --steps 5 --warmup 1 --no-hint-steps 10 || exit 1
done
cp gpurun_ab/lib_cur.so "$LIB"
echo "quick ab ok"
