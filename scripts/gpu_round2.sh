# Full GPU suite, then the round measurements (bench lines, rocprof kernel stats, PMC traffic).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
bash scripts/gpu_measure.sh || exit 1
bash scripts/pmc_traffic.sh || exit 1
cat profiles/pmc_traffic.json
