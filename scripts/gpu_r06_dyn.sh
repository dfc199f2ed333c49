#!/bin/bash
# Round 6: dynamic chunks in expand_fast (two static chunks per workgroup, then pulled from a counter)
# against static striding (gpurun_ab/lib_base.so, -DSR_DYN_CHUNKS=0): the whole GPU suite on the new
# build, then 2pc N=9 / 10 / 11, increment_lock N=11 and paxos C=6 alternately.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06dyn
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash scripts/gpu_lib_ab.sh r06dyn/n9 3 -- --steps 20 || exit 1
bash scripts/gpu_lib_ab.sh r06dyn/n10 2 -- --steps 5 --rm-count 10 || exit 1
bash scripts/gpu_lib_ab.sh r06dyn/n11 1 -- --steps 2 --warmup 1 --rm-count 11 || exit 1
bash scripts/gpu_lib_ab.sh r06dyn/il11 1 -- --steps 2 --warmup 1 --model increment_lock --threads 11 || exit 1
bash scripts/gpu_lib_ab.sh r06dyn/p6 2 -- --steps 5 --model paxos --clients 6 || exit 1
echo "dyn ok"
