#!/bin/bash
# Route-stage and filter knobs with self records at T=8 (2pc N=11), and the one-rank RCCL
# communicator's per-level kernel chain (kernel trace) with the direct exchange and with RCCL.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_route_knobs.sh 11 8 "SR_RSTAGE_WORDS=2048" "SR_RSTAGE_WORDS=3072" "SR_RSTAGE_WORDS=4096" "SR_RSTAGE_WORDS=2048 SR_FILTER_LOG2=10" "SR_RSTAGE_WORDS=2048 SR_FILTER_LOG2=11" "SR_RSTAGE_WORDS=2048 SR_SELF_RECORDS_MIN=0" || exit 1
mkdir -p gpurun_out/r03p
SR_DIRECT=1 bash scripts/ktrace.sh r03p/kt_rccl1_direct --mode rccl1 --steps 2 --warmup 1 --cpu-baseline 0 --config4-steps 0 || exit 1
SR_DIRECT=0 bash scripts/ktrace.sh r03p/kt_rccl1_a2a --mode rccl1 --steps 2 --warmup 1 --cpu-baseline 0 --config4-steps 0 || exit 1
echo done
