set -o pipefail
mkdir -p gpurun_out/px
for c in 3 6; do
  timeout -k 10 200 python -u bench.py --model paxos --clients $c --steps 10 --warmup 3 --cpu-baseline 0 --config4-steps 0 --no-hint-steps 0 > gpurun_out/px/p$c.json 2> gpurun_out/px/p$c.err || { tail -5 gpurun_out/px/p$c.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/px/p$c.json').read().strip().splitlines()[-1]); print('paxos $c', round(d['ms_per_step'],3), [round(x,1) for x in d['levels']['kernel_us']])"
done
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --cpu-baseline 0 --config4-steps 0 --no-hint-steps 0 > gpurun_out/px/b.json 2> gpurun_out/px/b.err || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/px/b.json').read().strip().splitlines()[-1]); print('2pc9', round(d['ms_per_step'],3), d['levels']['small_levels_ms'])"
