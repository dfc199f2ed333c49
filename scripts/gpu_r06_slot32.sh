#!/bin/bash
# Round 6: 32-bit quotient slots for one-word keys (2pc). Whole GPU suite on the new build, then
# the new library against the previous round's (gpurun_ab/lib_base.so) on 2pc N=9, and the slot
# width alone (SR_SLOT32=0: the same key in 8-byte quotient slots) at N=9/10/11.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06s
mkdir -p $O
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
bash scripts/gpu_lib_ab.sh r06s/lib 3 -- --steps 20 || exit 1
bash scripts/gpu_env_ab.sh r06s/env9 2 "SR_SLOT32=1" "SR_SLOT32=0" -- --steps 20 || exit 1
bash scripts/gpu_env_ab.sh r06s/env10 1 "SR_SLOT32=1" "SR_SLOT32=0" -- --rm-count 10 --steps 5 --warmup 1 || exit 1
bash scripts/gpu_env_ab.sh r06s/env11 1 "SR_SLOT32=1" "SR_SLOT32=0" -- --rm-count 11 --steps 2 --warmup 1 || exit 1
echo "r06 slot32 ok"
