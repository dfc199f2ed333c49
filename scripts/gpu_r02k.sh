#!/bin/bash
# rocprof kernel trace of the partitioned RCCL path on one rank (2pc N=9) and of the default bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02k_rccl1 -o run -- python3 bench.py --mode rccl1 --steps 5 --warmup 2 --config4-steps 0 --cpu-baseline 0 > gpurun_out/r02k_rccl1.json 2> gpurun_out/r02k_rccl1.err || { echo "rocprof rccl1 failed"; tail -20 gpurun_out/r02k_rccl1.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02k_bench -o run -- python3 bench.py --steps 10 --warmup 3 --config4-steps 0 --cpu-baseline 0 > gpurun_out/r02k_bench.json 2> gpurun_out/r02k_bench.err || { echo "rocprof bench failed"; tail -20 gpurun_out/r02k_bench.err; exit 1; }
find gpurun_out/r02k_rccl1 gpurun_out/r02k_bench -name "*.csv" | head -20
