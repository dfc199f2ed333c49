# One GPU call: rocprofv3 kernel-trace summaries (CSV) of the 2pc N=9 and paxos C=3 benches, then a
# visited-set load-factor sweep on 2pc N=9 (does a table that fits the 256 MB MALL pay?).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_2pc9 -o run -- python3 bench.py --steps 10 --warmup 3 --cpu-baseline 0 > gpurun_out/prof_2pc9.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_paxos3 -o run -- python3 bench.py --model paxos --clients 3 --steps 10 --warmup 3 --cpu-baseline 0 > gpurun_out/prof_paxos3.log 2>&1 || exit 1
: > gpurun_out/load_sweep.jsonl
for L in 0.25 0.5 0.62 0.75; do
  SR_TABLE_LOAD=$L timeout -k 10 120 python bench.py --steps 10 --warmup 3 --cpu-baseline 0 > gpurun_out/ls.json 2>/dev/null || exit 1
  python -c "import json,sys; d=json.load(open('gpurun_out/ls.json')); print(json.dumps({'table_load': $L, 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'cap': d['engine']['table_capacity'], 'avg_launch_ms': d['roofline']['avg_launch_ms']}))" >> gpurun_out/load_sweep.jsonl
done
cat gpurun_out/load_sweep.jsonl
find gpurun_out/prof_2pc9 gpurun_out/prof_paxos3 -name '*stats.csv'
