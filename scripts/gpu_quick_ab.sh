#!/bin/bash
# Quick GPU pass for an expand_fast probe-loop experiment: parity of the variants, timing A/B of
# SR_PROBE_BATCH settings, and their PMC summaries (scripts/pmc_variants.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-q}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_fingerprints.py tests/test_gpu_actor.py tests/test_gpu_explorer.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/fp.log 2>&1 || { tail -30 $O/fp.log; exit 1; }
tail -1 $O/fp.log
for pb in -4 -8; do
  SR_PROBE_BATCH=$pb timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/parity$pb.log 2>&1 || { tail -30 $O/parity$pb.log; exit 1; }
  tail -1 $O/parity$pb.log
done
bash scripts/gpu_env_ab.sh ${1:-q}/ab9 2 "SR_PROBE_BATCH=1" "SR_PROBE_BATCH=-4" "SR_PROBE_BATCH=-8" "SR_PROBE_BATCH=0" -- --steps 20 --warmup 3 || exit 1
bash scripts/gpu_env_ab.sh ${1:-q}/ab10 1 "SR_PROBE_BATCH=1" "SR_PROBE_BATCH=-4" "SR_PROBE_BATCH=-8" -- --steps 3 --warmup 1 --rm-count 10 || exit 1
bash scripts/gpu_env_ab.sh ${1:-q}/il10 1 "SR_PROBE_BATCH=1" "SR_PROBE_BATCH=-4" -- --steps 5 --warmup 1 --model increment_lock --threads 10 || exit 1
bash scripts/pmc_variants.sh $O/pmc "SR_PROBE_BATCH=1" "SR_PROBE_BATCH=-4" "SR_PROBE_BATCH=0" -- --rm-count 9 || exit 1
