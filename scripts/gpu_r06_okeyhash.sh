#!/bin/bash
# Round 6: config 4 with the owner key's partition by a multiplicative hash (lib_okeyhash, built with
# -DSR_OKEY_HASH=1) against fmix64 (the in-tree build): partitioned tests on the variant, then T = 8 / 4.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export SR_LIB_DIGEST_CHECK=0
LIB=stateright_amd/libstateright_gpu.so
cp $LIB gpurun_ab/lib_cur.so || exit 1
for T in 8 4; do bash scripts/gpu_okey_sweep.sh 11 $T "SR_V=cur" || exit 1; done
cp gpurun_ab/lib_okeyhash.so $LIB || exit 1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "partition or rank" > gpurun_out/okeyhash_tests.log 2>&1 || { tail -20 gpurun_out/okeyhash_tests.log; cp gpurun_ab/lib_cur.so $LIB; exit 1; }
tail -1 gpurun_out/okeyhash_tests.log
for T in 8 4; do bash scripts/gpu_okey_sweep.sh 11 $T "SR_V=okeyhash" || { cp gpurun_ab/lib_cur.so $LIB; exit 1; }; done
cp gpurun_ab/lib_cur.so $LIB
echo "okeyhash ok"
