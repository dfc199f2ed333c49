#!/bin/bash
# Counter passes comparing expand_route (2 virtual partitions) with expand_fast (one partition) on
# 2pc N=9; one rocprofv3 run per counter set (counters with --kernel-trace only).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/pmcr
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  for cfg in "virtual 1" "virtual 2"; do
    set -- $cfg
    timeout -s KILL 90 rocprofv3 --pmc $line --kernel-trace --output-format csv -d gpurun_out/pmcr/$1$2_p$i -o p -- python3 scripts/prof_partitioned.py $1 $2 9 2 > gpurun_out/pmcr/$1$2_p$i.log 2>&1 || { echo "fail $cfg pass $i"; tail -5 gpurun_out/pmcr/$1$2_p$i.log; exit 1; }
  done
  echo "pass $i ok"
done <<'PASSES'
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES
SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH
TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_ATOMIC_sum
PASSES
