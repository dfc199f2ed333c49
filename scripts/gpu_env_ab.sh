#!/bin/bash
# Alternating bench runs of 2pc N=9 (or other bench args) under different engine environment
# settings, for an A/B of an internal knob.
#   scripts/gpu_env_ab.sh <tag> <reps> "<env A>" "<env B>" [...] -- <bench args>
# e.g. scripts/gpu_env_ab.sh load 2 "" "SR_TABLE_LOAD=0.65" -- --steps 20
set -o pipefail
TAG=${1:?tag}; REPS=${2:?reps}; shift 2
ENVS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do ENVS+=("$1"); shift; done
[ "$1" = "--" ] && shift
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$TAG
mkdir -p "$O"
for r in $(seq 1 "$REPS"); do
    for i in "${!ENVS[@]}"; do
        label="e${i}_r${r}"
        env ${ENVS[$i]} timeout -k 10 200 python -u bench.py --cpu-baseline 0 --config4-steps 0 --no-hint-steps 0 "$@" > "$O/$label.json" 2> "$O/$label.err" || { tail -5 "$O/$label.err"; exit 1; }
        python3 -c "import json; d=json.loads(open('$O/$label.json').read().strip().splitlines()[-1]); l=d.get('levels') or {}; e=d.get('engine') or {}; print('[${ENVS[$i]}] r$r', round(d['ms_per_step'],4), 'big', round(l.get('big_levels_ms',0),4), 'small', round(l.get('small_levels_ms',0),4), 'gaps', round(l.get('gaps_ms',0),4), 'cap', e.get('table_capacity'))"
    done
done
echo "env ab ok"
