# A/B of per-check host-path knobs on the 2pc N=9 bench, alternating, 3 runs each:
#   single GPU: default | SR_TABLE_RECYCLE=0 (each check clears its visited set at its start)
#   gpurun -- bash scripts/gpu_sync_ab.sh <outdir>
set -o pipefail
out=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p $out
cd $GRAFT_REPO_ROOT
run() {  # name env... -- bench args
    local name=$1; shift
    env "$@" timeout -k 10 120 python3 bench.py --steps 30 --warmup 5 --config4-steps 0 --cpu-baseline 0 $BENCH_ARGS \
        > $out/$name.json 2> $out/$name.log || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],4))" $out/$name.json $name | tee -a $out/summary.txt
}
for i in 1 2 3; do
    BENCH_ARGS="" run default_$i SR_X=0
    BENCH_ARGS="" run norecycle_$i SR_TABLE_RECYCLE=0
done
for i in 1 2 3; do
    BENCH_ARGS="--mode rccl1" run rccl1_$i SR_X=0
done
