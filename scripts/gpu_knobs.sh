# One GPU call: expand_fast knob sweep on 2pc N=9 at the current code (duplicate filter size,
# probes in flight per lane, parents per wave). Each line: knobs, ms per full check, kernel avg.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/knob_sweep.jsonl
run() {
  env "$@" timeout -k 10 120 python bench.py --steps 10 --warmup 3 --cpu-baseline 0 > gpurun_out/k.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/k.json')); print(json.dumps({'knobs': '$*', 'ms_per_step': round(d['ms_per_step'],4), 'avg_launch_us': round(d['roofline']['avg_launch_ms']*1e3,2)}))" >> gpurun_out/knob_sweep.jsonl
}
run SR_NONE=1
for f in 0 8 10 11 12; do run SR_FILTER_LOG2=$f; done
run SR_PROBE_BATCH=2
for p in 4 5; do run SR_PPW_LOG2=$p; done
run SR_NONE=1
cat gpurun_out/knob_sweep.jsonl
