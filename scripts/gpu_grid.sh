# One GPU call: expand_fast grid capped (SR_GRID_MAX; the kernel grid-strides over the rest).
# 2pc N=9 bench per cap: ms per full check, level-loop span, summed expand-kernel time.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/grid_sweep.jsonl
run() {
  env "$@" timeout -k 10 120 python bench.py --steps 20 --warmup 3 --cpu-baseline 0 > gpurun_out/g.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/g.json')); r=d['roofline']; print(json.dumps({'knobs': '$*', 'ms_per_step': round(d['ms_per_step'],4), 'level_loop_ms': round(d['engine']['level_loop_sec']*1e3,4), 'kernel_ms_per_step': round(r['avg_launch_ms']*r['launches_per_step'],4)}))" >> gpurun_out/grid_sweep.jsonl
}
for rep in 1 2; do
  run SR_NONE=1
  for g in 1024 1536 2048 3072 6144; do run SR_GRID_MAX=$g; done
done
SR_GRID_MAX=1536 timeout -k 10 120 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "large_closed_form or paxos" --timeout 120 --timeout-method thread > gpurun_out/grid_tests.log 2>&1 || { tail -5 gpurun_out/grid_tests.log; exit 1; }
tail -1 gpurun_out/grid_tests.log
cat gpurun_out/grid_sweep.jsonl
