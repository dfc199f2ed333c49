#!/bin/bash
# Round 2: N=1 bench line, then the same bench under rocprofv3 kernel trace (stats summary).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py > gpurun_out/r02b_bench.json 2> gpurun_out/r02b_bench.err || { echo "bench failed"; tail -20 gpurun_out/r02b_bench.err; exit 1; }
cat gpurun_out/r02b_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02b_prof -o run -- python3 bench.py --cpu-baseline 0 > gpurun_out/r02b_prof_bench.json 2> gpurun_out/r02b_prof.err || { echo "rocprof failed"; tail -20 gpurun_out/r02b_prof.err; exit 1; }
find gpurun_out/r02b_prof -name "*stats*" | head
