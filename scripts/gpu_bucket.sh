set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/bk
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/bk/tests.log 2>&1 || { tail -40 gpurun_out/bk/tests.log; exit 1; }
tail -2 gpurun_out/bk/tests.log
for m in 0 150000; do SR_BUCKET_MIN=$m timeout -k 10 120 python3 scripts/gap_probe.py 9 noprof 2>&1 | grep -v amdgpu.ids || exit 1; done
for m in 0 150000; do SR_BUCKET_MIN=$m timeout -k 10 120 python3 scripts/gap_probe.py 10 noprof 2>&1 | grep -v amdgpu.ids || exit 1; done
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/bk/kt -o t -- python3 scripts/gap_probe.py 9 noprof > gpurun_out/bk/kt.log 2>&1 || exit 1
python3 scripts/ktrace_all.py gpurun_out/bk/kt/t_kernel_trace.csv
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --kernel-trace --output-format csv -d gpurun_out/bk/pmc3 -o p -- python3 scripts/gap_probe.py 9 noprof > gpurun_out/bk/pmc3.log 2>&1 || exit 1
python3 scripts/pmc_summary.py gpurun_out/bk
