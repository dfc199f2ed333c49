# Per-dispatch traces of a bench configuration under several SR_PPW_LOG2 values:
#   scripts/ktrace_env.sh "<ppw values>" <bench args...>
set -o pipefail
cd /tmp && export TMPDIR=/tmp
vals=$1; shift
for p in $vals; do
  out=$GRAFT_REPO_ROOT/gpurun_out/kt_ppw$p
  SR_PPW_LOG2=$p timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out -o trace -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 --cpu-baseline 0 "$@" > $out.log 2>&1 || exit 1
done
