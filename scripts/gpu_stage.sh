# One GPU call: expand_fast LDS stage size (blocks per CU) x duplicate-filter size, 2pc N=9 and paxos C=3.
# Variant libraries built by: hipcc ... -DSR_STAGE_WORDS=<S> -o variants/libsr_stage<S>.so engine.hip
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/stage_sweep.jsonl
run() {
  local model=$1; shift
  env "$@" timeout -k 10 120 python bench.py --model $model --steps 10 --warmup 3 --cpu-baseline 0 > gpurun_out/s.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/s.json')); print(json.dumps({'model': '$model', 'knobs': '$*', 'ms_per_step': round(d['ms_per_step'],4), 'avg_launch_us': round(d['roofline']['avg_launch_ms']*1e3,2)}))" >> gpurun_out/stage_sweep.jsonl
}
for m in 2pc paxos; do
  for lib in "" variants/libsr_stage768.so variants/libsr_stage512.so; do
    for f in 9 10; do
      if [ -n "$lib" ]; then run $m SR_LIB_PATH=$lib SR_FILTER_LOG2=$f; else run $m SR_FILTER_LOG2=$f; fi
    done
  done
done
cat gpurun_out/stage_sweep.jsonl
