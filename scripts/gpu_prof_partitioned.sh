#!/bin/bash
# Kernel traces of the partitioned search on one GPU: scripts/gpu_prof_partitioned.sh "<kind> <world>" ...
# (kind: local | virtual | rccl1; see scripts/prof_partitioned.py). Outputs: gpurun_out/pp/<kind><world>/
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/pp
for cfg in "$@"; do
  set -- $cfg
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pp/$1$2 -o t -- python3 scripts/prof_partitioned.py $1 $2 9 3 > gpurun_out/pp/$1$2.log 2>&1 || { echo "fail $cfg"; tail -5 gpurun_out/pp/$1$2.log; exit 1; }
done
echo done
