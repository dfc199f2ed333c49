#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_symmetry.py > gpurun_out/r02i.log 2>&1 || { echo "failed"; tail -50 gpurun_out/r02i.log; exit 1; }
grep -E "passed|failed" gpurun_out/r02i.log | tail -2
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r02i_tests.log 2>&1 || { echo "suite failed"; tail -40 gpurun_out/r02i_tests.log; exit 1; }
tail -2 gpurun_out/r02i_tests.log
