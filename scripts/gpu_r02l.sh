#!/bin/bash
# Side measurements: paxos C=3, increment_lock N=10/11/12, 2pc N=10 (one MI355X).
set -o pipefail
mkdir -p gpurun_out
run() { name=$1; shift; timeout -k 10 300 python -u bench.py --cpu-baseline 0 --config4-steps 0 "$@" > gpurun_out/r02l_$name.json 2> gpurun_out/r02l_$name.err || { echo "$name failed"; tail -20 gpurun_out/r02l_$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r02l_$name.json')); r=d['roofline']; print('$name', round(d['ms_per_step'],3), round(d['value']/1e9,3), 'probe_rate', r['probe_rate'] and round(r['probe_rate']/1e9,2), 'frac', round(r['frac'],4), 'levels', d['levels'] and (round(d['levels']['big_levels_ms'],3), round(d['levels']['small_levels_ms'],3), d['levels']['gaps_ms'] and round(d['levels']['gaps_ms'],3)))"; }
#run paxos3 --model paxos --clients 3 --steps 20
#run inclock10 --model increment_lock --threads 10 --steps 10
#run inclock11 --model increment_lock --threads 11 --steps 3 --warmup 1
run inclock12 --model increment_lock --threads 12 --steps 1 --warmup 1
run 2pc10 --rm-count 10 --steps 10
