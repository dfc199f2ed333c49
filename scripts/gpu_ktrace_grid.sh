set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/gc1
SR_GRID_MAX=1024 bash scripts/ktrace.sh gc1/kt_g1024 --steps 20 --warmup 3 --cpu-baseline 0 --config4-steps 0 --no-hint-steps 0 || exit 1
SR_GRID_MAX=2048 bash scripts/ktrace.sh gc1/kt_g2048 --steps 20 --warmup 3 --cpu-baseline 0 --config4-steps 0 --no-hint-steps 0 || exit 1
echo ok
