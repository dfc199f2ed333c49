set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/ktrace.sh ch2/kt_px3 --model paxos --clients 3 --steps 20 --warmup 3 --cpu-baseline 0 --config4-steps 0 --no-hint-steps 0 || exit 1
bash scripts/ktrace.sh ch2/kt_tp9 --steps 20 --warmup 3 --cpu-baseline 0 --config4-steps 0 --no-hint-steps 0 || exit 1
SR_CHAIN_MAX=0 bash scripts/ktrace.sh ch2/kt_px3_nc --model paxos --clients 3 --steps 20 --warmup 3 --cpu-baseline 0 --config4-steps 0 --no-hint-steps 0 || exit 1
echo ok
