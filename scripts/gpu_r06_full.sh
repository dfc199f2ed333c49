#!/bin/bash
# Round 6: whole GPU suite, then the default bench line and config 4 at T = 8 / 4 / 2.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r06full}
mkdir -p $O
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('bench', round(d['ms_per_step'],4), 'ms', round(d['value']/1e9,3), 'G/s', 'no_hint', d['no_hint']['ms_per_step'], d['no_hint']['vs_value'], 'config4', d.get('config4',{}).get('ms_per_step'), 'frac', d['roofline']['frac'], 'cpu', d['cpu_baseline']['value'])"
for T in 8 4 2; do bash scripts/gpu_okey_sweep.sh 11 $T "SR_X=0" || exit 1; done
echo "full ok"
