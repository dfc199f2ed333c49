#!/bin/bash
# Round 2: exact (quotient) visited set: increment_lock tests incl. N=12 on one GPU, then the suite.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu -k "increment_lock or inclock" tests/test_gpu_parity.py > gpurun_out/r02d_inclock.log 2>&1 || { echo "inclock tests failed"; tail -40 gpurun_out/r02d_inclock.log; exit 1; }
grep -E "passed|failed" gpurun_out/r02d_inclock.log | tail -3
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r02d_tests.log 2>&1 || { echo "suite failed"; tail -40 gpurun_out/r02d_tests.log; exit 1; }
tail -2 gpurun_out/r02d_tests.log
