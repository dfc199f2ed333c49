# Per-dispatch kernel trace of one bench configuration: scripts/ktrace.sh <outdir> <bench args...>
set -o pipefail
cd /tmp && export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/$1; shift
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o trace -- python3 $GRAFT_REPO_ROOT/bench.py "$@" > $out.log 2>&1
