#!/bin/bash
# Quick parity + timing of the single-GPU engine: the parity file, then the default bench (no CPU
# baseline, no config4) and a paxos bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_eventually.py > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --cpu-baseline 0 --config4-steps 0 > gpurun_out/ab_2pc.json 2> gpurun_out/ab_2pc.err || { tail -20 gpurun_out/ab_2pc.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/ab_2pc.json')); print('2pc9', round(d['ms_per_step'],3), d['levels'], d['roofline'].get('probe_rate'))"
timeout -k 10 200 python -u bench.py --model paxos --clients 3 --steps 10 --warmup 3 --cpu-baseline 0 --config4-steps 0 > gpurun_out/ab_paxos.json 2> gpurun_out/ab_paxos.err || { tail -20 gpurun_out/ab_paxos.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/ab_paxos.json')); print('paxos3', round(d['ms_per_step'],3))"
