#!/bin/bash
# Round 6: config 4 after the smaller default route stages and the single-hash route key: the
# partitioned / rank GPU tests, then T = 8, 4, 2 per-rank kernel time.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r06c4v}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "partition or dist or shm or rank or config4 or eventually or visit" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for T in 8 4 2; do bash scripts/gpu_okey_sweep.sh 11 $T "SR_X=0" || exit 1; done
echo "c4 verify ok"
