#!/bin/bash
# A/B of two builds of the engine library: gpurun_ab/lib_base.so (A) against the in-tree build (B),
# swapped into place alternately, bench.py with the given arguments.
#   scripts/gpu_lib_ab.sh <tag> <reps> [--parity <pytest -k expr>] -- <bench args>
set -o pipefail
TAG=${1:?tag}; REPS=${2:?reps}; shift 2
K=""
if [ "$1" = "--parity" ]; then K=$2; shift 2; fi
[ "$1" = "--" ] && shift
cd "$GRAFT_REPO_ROOT" || exit 1
export SR_LIB_DIGEST_CHECK=0  # lib_base.so is a build of older sources (see _native.check_digest)
O=gpurun_out/$TAG
mkdir -p "$O"
LIB=stateright_amd/libstateright_gpu.so
cp "$LIB" gpurun_ab/lib_new.so || exit 1
if [ -n "$K" ]; then
    timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "$K" --timeout 120 --timeout-method thread > "$O/parity.log" 2>&1 || { tail -30 "$O/parity.log"; exit 1; }
    tail -1 "$O/parity.log"
fi
for r in $(seq 1 "$REPS"); do
    for v in base new; do
        cp "gpurun_ab/lib_$v.so" "$LIB" || exit 1
        timeout -k 10 200 python -u bench.py --cpu-baseline 0 --config4-steps 0 --no-hint-steps 0 "$@" > "$O/${v}_$r.json" 2> "$O/${v}_$r.err" || { tail -5 "$O/${v}_$r.err"; cp gpurun_ab/lib_new.so "$LIB"; exit 1; }
        python3 -c "import json; d=json.loads(open('$O/${v}_$r.json').read().strip().splitlines()[-1]); l=d.get('levels',{}); print('$v r$r', round(d['ms_per_step'],4), 'small', round(l.get('small_levels_ms',0),4), 'gaps', round(l.get('gaps_ms',0),4), 'unique', d['value']*d['ms_per_step']/1e3)"
    done
done
cp gpurun_ab/lib_new.so "$LIB"
echo "lib ab ok"
