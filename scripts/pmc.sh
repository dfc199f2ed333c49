#!/bin/bash
# PMC passes (one rocprofv3 run each, counters only with --kernel-trace/--stats, per the pool rules).
set -e
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmc}
mkdir -p $OUT
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $line --kernel-trace --output-format csv -d $OUT/p$i -o p$i -- python3 scripts/prof_driver.py > $OUT/p$i.log 2>&1
  echo "pass $i ok: $line"
done <<'PASSES'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_VALU
TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum
FETCH_SIZE
WRITE_SIZE TCC_EA0_ATOMIC_sum
TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum
TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_TAG_STALL_sum
GRBM_GUI_ACTIVE TA_BUSY_avr SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INST_LEVEL_VMEM
PASSES
