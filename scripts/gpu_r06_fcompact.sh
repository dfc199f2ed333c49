#!/bin/bash
# Round 6: the compact LDS filter (4-byte entries, twice the entries in the same LDS, where exact:
# 2pc N <= 9) against 8-byte entries (SR_FILTER_COMPACT=0): the 2pc / small-model GPU tests, then
# 2pc N=9 alternately, with the per-level probe counts of the counting pass.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06fc
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "2pc or two_phase or growth or probe or doubling or rehash or linear or clock or puzzle or plugin or symmetry" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash scripts/gpu_env_ab.sh r06fc/n9 4 "SR_FILTER_COMPACT=0" "SR_X=0" -- --steps 20 || exit 1
bash scripts/gpu_env_ab.sh r06fc/n9f11 2 "SR_FILTER_LOG2=10" -- --steps 20 || exit 1
echo "fcompact ok"
