#!/bin/bash
# The launcher path of bench.py on the one-GPU box: torch.distributed.run with one rank, the RCCL
# partitioned path bootstrapped through Communicator.from_env (file rendezvous), config4 included.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --mode rccl1 --cpu-baseline 0 --steps 5 > gpurun_out/r02o.json 2> gpurun_out/r02o.err || { echo "launcher run failed"; tail -30 gpurun_out/r02o.err; exit 1; }
python3 -c "
import json
lines=[l for l in open('gpurun_out/r02o.json') if l.startswith('{')]
d=json.loads(lines[-1]); print(len(lines), d['config'], d['ms_per_step'], d.get('config4'))"
