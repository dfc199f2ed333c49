#!/bin/bash
# Bench (2pc N=9, no CPU baseline/config4) under each environment setting given as an argument:
#   scripts/gpu_env_sweep.sh "SR_GRID_MAX=1536" "SR_GRID_MAX=3072" ...
# (BENCH_ARGS adds bench.py arguments, e.g. BENCH_ARGS="--rm-count 11 --steps 5")
set -o pipefail
mkdir -p gpurun_out/sweep
for kv in "$@"; do
  name=$(echo "$kv $BENCH_ARGS" | tr ' =/-' '____')
  env $kv timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 --cpu-baseline 0 --config4-steps 0 --no-hint-steps 0 $BENCH_ARGS > gpurun_out/sweep/$name.json 2> gpurun_out/sweep/$name.err || { echo "fail $kv"; tail -5 gpurun_out/sweep/$name.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/sweep/$name.json')); l=d['levels']; print('$kv', round(d['ms_per_step'],3), 'big', round(l['big_levels_ms'],3), 'small', round(l['small_levels_ms'],3), 'gaps', round(l['gaps_ms'],3))"
done
