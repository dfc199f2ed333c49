set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/gp
timeout -k 10 120 python3 scripts/gap_probe.py 9 both || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gp/noprof -o t -- python3 scripts/gap_probe.py 9 noprof > gpurun_out/gp/noprof.log 2>&1 || exit 1
python3 scripts/gaps.py gpurun_out/gp/noprof/t_kernel_trace.csv
