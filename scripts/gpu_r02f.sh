#!/bin/bash
# Round 2: suite, N=1 bench (with config4), partitioned RCCL path rehearsal on one rank.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r02f_tests.log 2>&1 || { echo "suite failed"; tail -40 gpurun_out/r02f_tests.log; exit 1; }
tail -2 gpurun_out/r02f_tests.log
timeout -k 10 300 python -u bench.py --cpu-baseline 0 > gpurun_out/r02f_bench.json 2> gpurun_out/r02f_bench.err || { echo "bench failed"; tail -20 gpurun_out/r02f_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r02f_bench.json')); print(d['ms_per_step'], d['value']/1e9, d['config4'])"
timeout -k 10 300 python -u bench.py --cpu-baseline 0 --mode rccl1 --config4-steps 0 > gpurun_out/r02f_rccl1.json 2> gpurun_out/r02f_rccl1.err || { echo "rccl1 failed"; tail -20 gpurun_out/r02f_rccl1.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r02f_rccl1.json')); print('rccl1', d['ms_per_step'], d['value']/1e9, d['engine'])"
