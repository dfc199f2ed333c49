#!/bin/bash
# A/B over several builds of the engine library: gpurun_ab/lib_<name>.so for each name, and "new" for
# the in-tree build, swapped into place in turn, bench.py with the given arguments.
#   scripts/gpu_libs_ab.sh <tag> <reps> <name> ... -- <bench args>
set -o pipefail
TAG=${1:?tag}; REPS=${2:?reps}; shift 2
NAMES=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do NAMES+=("$1"); shift; done
[ "$1" = "--" ] && shift
cd "$GRAFT_REPO_ROOT" || exit 1
export SR_LIB_DIGEST_CHECK=0  # the variants are builds of other sources (see _native.check_digest)
O=gpurun_out/$TAG
mkdir -p "$O"
LIB=stateright_amd/libstateright_gpu.so
cp "$LIB" gpurun_ab/lib_new.so || exit 1
for r in $(seq 1 "$REPS"); do
    for v in "${NAMES[@]}"; do
        cp "gpurun_ab/lib_$v.so" "$LIB" || exit 1
        timeout -k 10 200 python -u bench.py --cpu-baseline 0 --config4-steps 0 --no-hint-steps 0 "$@" > "$O/${v}_$r.json" 2> "$O/${v}_$r.err" || { tail -5 "$O/${v}_$r.err"; cp gpurun_ab/lib_new.so "$LIB"; exit 1; }
        python3 -c "import json; d=json.loads(open('$O/${v}_$r.json').read().strip().splitlines()[-1]); l=d.get('levels',{}); print('$v r$r', round(d['ms_per_step'],4), 'big', round(l.get('big_levels_ms',0),4), 'small', round(l.get('small_levels_ms',0),4), 'unique', d['value']*d['ms_per_step']/1e3)"
    done
done
cp gpurun_ab/lib_new.so "$LIB"
echo "libs ab ok"
