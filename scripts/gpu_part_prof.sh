set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_p2 -o run -- python3 scripts/trace_partitioned.py 9 2 > gpurun_out/prof_p2.log 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rccl -o run -- python3 scripts/trace_partitioned.py 9 0 > gpurun_out/prof_rccl.log 2>&1
find gpurun_out/prof_p2 gpurun_out/prof_rccl -name "*stats*"
