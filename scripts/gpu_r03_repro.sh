#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03s
mkdir -p $O
SR_DIST_TRACE=1 SR_PEER_TIMEOUT_MS=3000 timeout -k 10 300 python -u -m pytest tests/test_gpu_dist_ranks.py -x -v -s -k "repeated_checks_same_ranks" --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|sr-direct" $O/tests.log | head -40
exit $rc
