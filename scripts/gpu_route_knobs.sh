#!/bin/bash
# Kernel time of the partitioned search (T virtual partitions on one GPU) under route-kernel knobs:
#   scripts/gpu_route_knobs.sh <N> <T> "<ENV=V ...>" ...      (one quoted env set per point; "" = defaults)
# Each point: rocprofv3 --kernel-trace --stats over 2 checks after one warmup; prints the top kernels.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/knobs
N=$1; T=$2; shift 2
i=0
for envs in "$@"; do
  i=$((i + 1))
  d=gpurun_out/knobs/n${N}_t${T}_$i
  echo "== $envs"
  env $envs timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o t -- python3 scripts/prof_partitioned.py virtual $T $N 2 > $d.log 2>&1 || { echo "fail $envs"; tail -5 $d.log; exit 1; }
  tail -1 $d.log
  python3 - "$d/t_kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:5]:
    print(f"  {r['Name'][:50]:50s} calls {r['Calls']:>6s} total/check {float(r['TotalDurationNs'])/3e6:9.2f} ms avg {float(r['AverageNs'])/1e3:8.1f} us")
PY
done
