# One GPU call: the default expand grid cap (two device residencies) against explicit caps, 2pc N=9
# and paxos C=3, then the full GPU parity suite with the default cap.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/gridcap.jsonl
run() {
  local model=$1; shift
  env "$@" timeout -k 10 120 python bench.py --model $model --steps 20 --warmup 3 --cpu-baseline 0 > gpurun_out/gc.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/gc.json')); print(json.dumps({'model': '$model', 'knobs': '$*', 'ms_per_step': round(d['ms_per_step'],4), 'avg_launch_us': round(d['roofline']['avg_launch_ms']*1e3,2)}))" >> gpurun_out/gridcap.jsonl
}
for rep in 1 2; do
  for m in 2pc paxos; do
    run $m SR_NONE=1
    run $m SR_GRID_MAX=3072
    run $m SR_GRID_MAX=1000000000
  done
done
cat gpurun_out/gridcap.jsonl
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
