#!/bin/bash
# Quick GPU pass for an expand_fast experiment: parity under the knob, timing A/B of settings, and
# their PMC summaries (scripts/pmc_variants.sh). Usage: scripts/gpu_quick_ab.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-q}
O=gpurun_out/$T
mkdir -p $O
SR_XCD_MAP=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/parity_xcd.log 2>&1 || { tail -30 $O/parity_xcd.log; exit 1; }
tail -1 $O/parity_xcd.log
bash scripts/gpu_env_ab.sh $T/ab9 2 "" "SR_XCD_MAP=1" "SR_FILTER_LOG2=10" "SR_FILTER_LOG2=11" "SR_XCD_MAP=1 SR_FILTER_LOG2=10" "SR_XCD_MAP=1 SR_PROBE_BATCH=-4" -- --steps 20 --warmup 3 || exit 1
bash scripts/gpu_env_ab.sh $T/ab10 1 "" "SR_XCD_MAP=1" "SR_PROBE_BATCH=-4" "SR_XCD_MAP=1 SR_PROBE_BATCH=-4" "SR_FILTER_LOG2=10" -- --steps 3 --warmup 1 --rm-count 10 || exit 1
bash scripts/gpu_env_ab.sh $T/ab11 1 "" "SR_XCD_MAP=1" "SR_PROBE_BATCH=-4" -- --steps 2 --warmup 1 --rm-count 11 || exit 1
bash scripts/pmc_variants.sh $O/pmc "" "SR_XCD_MAP=1" "SR_FILTER_LOG2=10" -- --rm-count 9 || exit 1
