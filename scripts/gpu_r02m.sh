#!/bin/bash
# PMC pass over the paxos C=3 bench: instruction mix of the expand kernel (one counter pass).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --output-format csv -d gpurun_out/r02m_pmc -o run -- python3 bench.py --model paxos --clients 3 --steps 2 --warmup 1 --config4-steps 0 --cpu-baseline 0 > gpurun_out/r02m.json 2> gpurun_out/r02m.err || { echo "pmc failed"; tail -20 gpurun_out/r02m.err; exit 1; }
find gpurun_out/r02m_pmc -name "*.csv"
