# A/B of the visited-set recycle (SR_TABLE_RECYCLE: a freed checker's table is cleared behind it on
# the device, the next check takes it clean) on the 2pc N=9 bench, alternating, 3 runs each.
#   gpurun -- bash scripts/gpu_recycle_ab.sh <outdir>
set -o pipefail
out=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p $out
cd $GRAFT_REPO_ROOT
for i in 1 2 3; do
    for r in 0 1; do
        SR_TABLE_RECYCLE=$r timeout -k 10 120 python3 bench.py --steps 30 --warmup 5 --config4-steps 0 --cpu-baseline 0 \
            > $out/r${r}_$i.json 2> $out/r${r}_$i.log || exit 1
        python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[1].split('/')[-1], round(d['ms_per_step'],4))" $out/r${r}_$i.json | tee -a $out/summary.txt
    done
done
