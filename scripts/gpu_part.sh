set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_partitioned.py -x -q --timeout 120 --timeout-method thread > gpurun_out/part_tests.log 2>&1 || { tail -30 gpurun_out/part_tests.log; exit 1; }
tail -2 gpurun_out/part_tests.log
echo "== new"; timeout -k 10 120 python -u scripts/time_partitioned.py 9 2>&1 | grep -v "version\|Hostname\|path"
timeout -k 10 60 python -u scripts/trace_partitioned.py 9 2 > gpurun_out/trace_p2.log 2>&1
timeout -k 10 60 python -u scripts/trace_partitioned.py 9 0 > gpurun_out/trace_rccl.log 2>&1
