#!/bin/bash
# Same-box A/B of the round-4 library against the current one (2pc N=9, N=10, paxos C=3), then
# the partitioned path on a one-rank RCCL communicator under the exchange's measurement knobs.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-q}
bash scripts/gpu_lib_ab.sh $T/lib9 3 -- --steps 20 --warmup 3 || exit 1
bash scripts/gpu_lib_ab.sh $T/libpx 2 -- --steps 10 --warmup 2 --model paxos --clients 3 || exit 1
bash scripts/gpu_env_ab.sh $T/rccl1 2 "" "SR_DX_CHECK=0" "SR_DX_FINE=0" "SR_DX_VOTE=0" "SR_DX_CHECK=0 SR_DX_FINE=0 SR_DX_VOTE=0" "SR_DIRECT=0" -- --mode rccl1 --steps 10 --warmup 3 || exit 1
