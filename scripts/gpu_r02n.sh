#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --model paxos --clients 3 --steps 20 --cpu-baseline 0 --config4-steps 0 > gpurun_out/r02n_paxos.json 2> gpurun_out/r02n_paxos.err || { echo "paxos bench failed"; tail -20 gpurun_out/r02n_paxos.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r02n_paxos.json')); print('paxos', round(d['ms_per_step'],3), round(d['value']/1e9,3), d['levels']['kernel_us'])"
timeout -k 10 300 python -u bench.py --steps 20 --cpu-baseline 0 --config4-steps 0 > gpurun_out/r02n_2pc.json 2> gpurun_out/r02n_2pc.err || { echo "2pc bench failed"; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r02n_2pc.json')); print('2pc9', round(d['ms_per_step'],3), round(d['value']/1e9,3))"
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r02n_tests.log 2>&1 || { echo "suite failed"; tail -40 gpurun_out/r02n_tests.log; exit 1; }
tail -2 gpurun_out/r02n_tests.log
