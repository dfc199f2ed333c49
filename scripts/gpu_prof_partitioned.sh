#!/bin/bash
# Kernel traces of the partitioned search on one GPU:
#   scripts/gpu_prof_partitioned.sh <N> "<kind> <world>" ...
# (kind: local | virtual | rccl1; see scripts/prof_partitioned.py). Outputs: gpurun_out/pp/<kind><world>_n<N>/
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/pp
N=$1; shift
for cfg in "$@"; do
  set -- $cfg
  d=gpurun_out/pp/$1$2_n$N
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o t -- python3 scripts/prof_partitioned.py $1 $2 $N 2 > $d.log 2>&1 || { echo "fail $cfg"; tail -5 $d.log; exit 1; }
  python3 - "$d/t_kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:6]:
    print(f"  {r['Name'][:60]:60s} calls {r['Calls']:>6s} total {float(r['TotalDurationNs'])/1e6:9.2f} ms avg {float(r['AverageNs'])/1e3:8.1f} us")
PY
done
echo done
