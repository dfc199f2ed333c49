#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/n11_probe.py 11 > gpurun_out/n11_flush.log 2>&1 || { tail -20 gpurun_out/n11_flush.log; exit 1; }
grep "^check" gpurun_out/n11_flush.log
timeout -k 10 300 python -u bench.py --cpu-baseline 0 > gpurun_out/r02g_bench.json 2> gpurun_out/r02g_bench.err || { echo "bench failed"; tail -20 gpurun_out/r02g_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r02g_bench.json')); print(d['ms_per_step'], d['value']/1e9, d['config4']['ms_per_step'], d['levels']['kernel_us'])"
timeout -k 10 300 python -u bench.py --cpu-baseline 0 --mode rccl1 --config4-steps 0 > gpurun_out/r02g_rccl1.json 2> gpurun_out/r02g_rccl1.err || { echo "rccl1 failed"; tail -20 gpurun_out/r02g_rccl1.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r02g_rccl1.json')); print('rccl1', d['ms_per_step'], d['value']/1e9, d['engine'])"
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r02g_tests.log 2>&1 || { echo "suite failed"; tail -40 gpurun_out/r02g_tests.log; exit 1; }
tail -2 gpurun_out/r02g_tests.log
