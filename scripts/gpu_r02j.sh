#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -k "multi_level" tests/test_gpu_parity.py > gpurun_out/r02j_multi.log 2>&1 || { echo "multi tests failed"; tail -60 gpurun_out/r02j_multi.log; exit 1; }
grep -E "passed|failed" gpurun_out/r02j_multi.log | tail -2
for m in 0 8192 32768; do
  SR_MULTI_MAX_N=$m timeout -k 10 300 python -u bench.py --cpu-baseline 0 --config4-steps 0 --steps 20 > gpurun_out/r02j_bench_$m.json 2> gpurun_out/r02j_bench_$m.err || { echo "bench $m failed"; tail -20 gpurun_out/r02j_bench_$m.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r02j_bench_$m.json')); print('$m', round(d['ms_per_step'],3), round(d['value']/1e9,3), d['levels']['kernel_us'][:12], d['levels']['gaps_ms'])"
done
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r02j_tests.log 2>&1 || { echo "suite failed"; tail -40 gpurun_out/r02j_tests.log; exit 1; }
tail -2 gpurun_out/r02j_tests.log
