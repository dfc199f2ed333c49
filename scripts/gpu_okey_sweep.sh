#!/bin/bash
# Owner-key / route-kernel sweep of BASELINE config 4 (2pc N, T virtual partitions on one GPU):
#   scripts/gpu_okey_sweep.sh <N> <T> "<VAR=value ...>" ...   (e.g. "SR_OWNER_RMS=4 SR_LSTAGE_WORDS=512";
#   SR_OWNER_RMS=0 owns states by fingerprint)
# Per setting: rocprofv3 kernel trace of one warmup + one timed check, then per-partition balance.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/okey
N=$1; T=$2; shift 2
for setting in "$@"; do
  tag=$(echo "$setting" | tr ' =' '_-')
  d=gpurun_out/okey/n${N}_t${T}_$tag
  env $setting timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o t -- \
    python3 scripts/prof_partitioned.py virtual $T $N 1 > $d.log 2>&1 || { echo "fail $setting"; tail -5 $d.log; exit 1; }
  echo "== $setting: $(grep '^ok' $d.log)"
  python3 scripts/partition_balance.py $d/t_kernel_trace.csv $T 2 || exit 1
done
echo done
