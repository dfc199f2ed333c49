#!/bin/bash
# Round 6: memory-side read latency (Little), reads in flight and UTCL1 misses of expand_fast's big
# levels with 32-bit quotient slots (2pc N=9 and N=11), and N=9 with the key in 8-byte slots.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/pmc_inflight.sh > gpurun_out/r06_pmc_inflight.txt 2>&1 || { tail -20 gpurun_out/r06_pmc_inflight.txt; exit 1; }
cat gpurun_out/r06_pmc_inflight.txt
bash scripts/pmc_variants.sh gpurun_out/r06_pmc_var "SR_SLOT32=1" "SR_SLOT32=0" -- > gpurun_out/r06_pmc_var.txt 2>&1 || { tail -20 gpurun_out/r06_pmc_var.txt; exit 1; }
cat gpurun_out/r06_pmc_var.txt
