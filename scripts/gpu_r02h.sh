#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_explorer.py tests/test_gpu_eventually.py > gpurun_out/r02h.log 2>&1 || { echo "failed"; tail -50 gpurun_out/r02h.log; exit 1; }
grep -E "passed|failed" gpurun_out/r02h.log | tail -2
