set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/q1
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_actor.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/q1/parity.log 2>&1 || { tail -30 gpurun_out/q1/parity.log; exit 1; }
tail -2 gpurun_out/q1/parity.log
bash scripts/gpu_env_ab.sh q1/ab9 3 "SR_PROBE_BATCH=1" "SR_PROBE_BATCH=0" -- --steps 20 --warmup 3 || exit 1
bash scripts/gpu_env_ab.sh q1/ab10 1 "SR_PROBE_BATCH=1" "SR_PROBE_BATCH=0" -- --steps 3 --warmup 1 --rm-count 10 || exit 1
bash scripts/gpu_env_ab.sh q1/px3 2 "SR_PROBE_BATCH=1" "SR_PROBE_BATCH=0" -- --steps 10 --warmup 2 --model paxos --clients 3 || exit 1
bash scripts/gpu_env_ab.sh q1/il10 1 "SR_PROBE_BATCH=1" "SR_PROBE_BATCH=0" -- --steps 5 --warmup 1 --model increment_lock --threads 10 || exit 1
