#!/bin/bash
# Round 6: paxos with the branch-free server handler (px::server_on_msg_sel) against the previous
# build (gpurun_ab/lib_base.so): actor/paxos GPU parity first, then C=3 and C=6 alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r06px}
bash scripts/gpu_lib_ab.sh $T/c3 3 --parity "paxos or actor or single or abd or ping or register or fingerprint" -- --model paxos --clients 3 --steps 200 --warmup 5 || exit 1
bash scripts/gpu_lib_ab.sh $T/c6 2 -- --model paxos --clients 6 --steps 30 --warmup 2 || exit 1
echo "paxos ab ok"
