#!/bin/bash
# Instruction mix, occupancy and memory-level parallelism of expand_fast's big levels (launches of
# >= 100 us) under several engine settings, two PMC passes per setting (counters only, with
# --kernel-trace): A = SQ instruction and wave counters, B = memory-side read requests and their
# per-cycle level. Summarised by scripts/pmc_variants.py.
#   scripts/pmc_variants.sh <outdir> "<env A>" "<env B>" ... -- <bench args>
set -o pipefail
O=${1:?outdir}; shift
ENVS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do ENVS+=("$1"); shift; done
[ "$1" = "--" ] && shift
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p "$O"
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
B="TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_ATOMIC_sum GRBM_GUI_ACTIVE"
for i in "${!ENVS[@]}"; do
  for p in A B; do
    env ${ENVS[$i]} timeout -s KILL 120 rocprofv3 --pmc ${!p} --kernel-trace --output-format csv -d "$O/v${i}_$p" -o p -- \
        python3 bench.py --steps 1 --warmup 1 --cpu-baseline 0 --config4-steps 0 --no-hint-steps 0 "$@" > "$O/v${i}_$p.log" 2>&1 \
        || { echo "variant $i pass $p failed"; tail -3 "$O/v${i}_$p.log"; exit 1; }
  done
done
python3 scripts/pmc_variants.py "$O" "${ENVS[@]}"
