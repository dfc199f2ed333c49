#!/bin/bash
# Last GPU pass of a round at the committed sources: the whole -m gpu suite, the PMC request
# ceilings and per-config traffic stamped with the current source digest (scripts/gpu_roofline.sh),
# then the default bench line, which reads those PMC files (copy gpurun_out/roofline/pmc_*.json
# into profiles/ before the bench so the line carries the traffic).
#   scripts/gpu_finish.sh <tag>
set -o pipefail
TAG=${1:?tag}
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/gpu_tests.log" 2>&1 || { tail -30 "$O/gpu_tests.log"; exit 1; }
tail -1 "$O/gpu_tests.log"
bash scripts/gpu_roofline.sh || exit 1
cp gpurun_out/roofline/pmc_ceiling.json gpurun_out/roofline/pmc_traffic.json profiles/ || exit 1
timeout -k 10 400 python -u bench.py > "$O/bench.json" 2> "$O/bench.err" || { tail -5 "$O/bench.err"; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'], d['roofline']['frac'], d['roofline']['traffic'], d['roofline']['pmc'])"
echo "finish ok"
