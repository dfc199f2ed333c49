# A/B: in-tree library vs build/old/libstateright_gpu.so (partitioned timings + 2pc / paxos bench)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for lib in stateright_amd/libstateright_gpu.so build/old/libstateright_gpu.so; do
  echo "== $lib"
  SR_LIB_PATH=$lib timeout -k 10 120 python -u scripts/time_partitioned.py 9 2>&1 | grep -v "version\|Hostname\|path" || exit 1
  SR_LIB_PATH=$lib timeout -k 10 120 python bench.py --steps 10 --warmup 3 --cpu-baseline 0 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('2pc9', round(d['value']/1e9,3), 'G/s', round(d['ms_per_step'],3), 'ms')" || exit 1
  SR_LIB_PATH=$lib timeout -k 10 120 python bench.py --model paxos --steps 10 --warmup 3 --cpu-baseline 0 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('paxos3', round(d['value']/1e9,3), 'G/s', round(d['ms_per_step'],3), 'ms')" || exit 1
done
