set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/gaps
for p in 0 1; do
  SR_PIPELINE=$p timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gaps/p$p -o t -- python3 bench.py --steps 2 --warmup 1 --cpu-baseline 0 > gpurun_out/gaps/p$p.log 2>&1 || exit 1
  python3 scripts/gaps.py gpurun_out/gaps/p$p/t_kernel_trace.csv
done
