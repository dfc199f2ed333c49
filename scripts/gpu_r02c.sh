#!/bin/bash
# Round 2: the whole GPU suite, then the N=1 bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r02c_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r02c_tests.log; exit 1; }
tail -3 gpurun_out/r02c_tests.log
timeout -k 10 300 python -u bench.py --cpu-baseline 0 > gpurun_out/r02c_bench.json 2> gpurun_out/r02c_bench.err || { echo "bench failed"; tail -20 gpurun_out/r02c_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r02c_bench.json')); print(d['ms_per_step'], d['value']/1e9, d['levels']['kernel_us'], d['levels']['gaps_ms'])"
