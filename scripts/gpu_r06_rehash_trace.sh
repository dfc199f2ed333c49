#!/bin/bash
# Round 6: kernel traces of unhinted increment_lock N=11 and 2pc N=10 with growth by ranges.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
SR_REHASH_RANGES=1 bash scripts/ktrace.sh r06rht_il --model increment_lock --threads 11 --steps 1 --warmup 1 --no-hint-steps 2 --cpu-baseline 0 --config4-steps 0 || exit 1
SR_REHASH_RANGES=1 bash scripts/ktrace.sh r06rht_2pc10 --rm-count 10 --steps 1 --warmup 1 --no-hint-steps 2 --cpu-baseline 0 --config4-steps 0 || exit 1
echo "trace ok"
