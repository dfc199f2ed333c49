#!/bin/bash
# Occupancy and memory-level parallelism of expand_fast's big levels (2pc N=9 and N=11, single GPU):
# one PMC pass per configuration with resident wave-cycles, the VMEM instruction level (outstanding
# vector-memory instructions summed per cycle), L1->L2 read requests and their latency, and the
# memory-side read requests. Summarised per dispatch >= 100 us by scripts/pmc_inflight.py.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/pmc_inflight
mkdir -p $O
for n in 9 11; do
  timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM \
      TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCC_EA0_RDREQ_sum --kernel-trace --output-format csv \
      -d $O/n$n -o p -- python3 bench.py --rm-count $n --steps 1 --warmup 1 --cpu-baseline 0 --config4-steps 0 \
      --no-hint-steps 0 > $O/n$n.log 2>&1 || { echo "n$n failed"; tail -3 $O/n$n.log; exit 1; }
done
python3 scripts/pmc_inflight.py $O
