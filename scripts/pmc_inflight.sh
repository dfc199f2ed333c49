#!/bin/bash
# Occupancy, memory-level parallelism and address translation of expand_fast's big levels (2pc N=9
# and N=11, single GPU), three PMC passes per configuration (rocprofv3 collects no counter across
# passes): A resident waves and outstanding vector-memory instructions (per-cycle levels),
# B memory-side read requests and their per-cycle level (requests in flight beyond L2),
# C L1 address translation (UTCL1 hits, misses, stalls). Summarised by scripts/pmc_inflight.py.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/pmc_inflight
mkdir -p $O
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LEVEL_WAVES SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
B="TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE"
C="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_INFLIGHT_MAX_sum TCP_UTCL1_STALL_MULTI_MISS_sum GRBM_GUI_ACTIVE"
for n in 9 11; do
  for p in A B C; do
    timeout -s KILL 180 rocprofv3 --pmc ${!p} --kernel-trace --output-format csv -d $O/n${n}_$p -o p -- python3 bench.py \
        --rm-count $n --steps 1 --warmup 1 --cpu-baseline 0 --config4-steps 0 --no-hint-steps 0 > $O/n${n}_$p.log 2>&1 \
        || { echo "n$n pass $p failed"; tail -3 $O/n${n}_$p.log; exit 1; }
  done
done
python3 scripts/pmc_inflight.py $O
