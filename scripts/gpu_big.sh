set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "large_closed_form or fifo_matches_fast" > gpurun_out/big_tests.log 2>&1 || { tail -30 gpurun_out/big_tests.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/big_tests.log | tail -15
