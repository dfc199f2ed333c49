#!/bin/bash
# Quick GPU timing of the register models (paxos C=3 and 6, single-copy register C=4) and the
# headline 2pc N=9 (no CPU baseline, no side legs): one line each.
set -o pipefail
mkdir -p gpurun_out/px
run() {  # name, bench args
    local name=$1; shift
    timeout -k 10 200 python -u bench.py "$@" --cpu-baseline 0 --config4-steps 0 --no-hint-steps 0 > gpurun_out/px/$name.json 2> gpurun_out/px/$name.err || { tail -5 gpurun_out/px/$name.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/px/$name.json').read().strip().splitlines()[-1]); l=d.get('levels') or {}; print('$name', round(d['ms_per_step'],3), 'small', round(l.get('small_levels_ms', 0), 3), [round(x,1) for x in l.get('kernel_us', [])][:40])"
}
run paxos3 --model paxos --clients 3 --steps 10 --warmup 3
run paxos6 --model paxos --clients 6 --steps 5 --warmup 2
run single_copy4 --model single_copy --clients 4 --steps 10 --warmup 3
run 2pc9 --steps 20 --warmup 3
