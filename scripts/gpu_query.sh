# One GPU call: does the host's periodic hipStreamQuery (wait_publish) cost inter-level gaps?
# 2pc N=9 bench per knob: ms per full check, level-loop span, summed expand-kernel time.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/query_sweep.jsonl
run() {
  env "$@" timeout -k 10 120 python bench.py --steps 20 --warmup 3 --cpu-baseline 0 > gpurun_out/q.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/q.json')); r=d['roofline']; print(json.dumps({'knobs': '$*', 'ms_per_step': round(d['ms_per_step'],4), 'level_loop_ms': round(d['engine']['level_loop_sec']*1e3,4), 'kernel_ms_per_step': round(r['avg_launch_ms']*r['launches_per_step'],4)}))" >> gpurun_out/query_sweep.jsonl
}
for rep in 1 2; do
  run SR_QUERY_LOG2=12
  run SR_QUERY_LOG2=22
  run SR_QUERY_LOG2=8
  run SR_PIPELINE=0
done
cat gpurun_out/query_sweep.jsonl
