#!/bin/bash
# Register, LDS and occupancy figures of the engine's kernels (the compiler's kernel-resource-usage
# remarks), device code only, for one registry family:
#   scripts/kernel_resources.sh <reg_*.hip> [kernel-name regex]
set -e
cd "$(dirname "$0")/.."
SRC=${1:?reg_*.hip}
PAT=${2:-expand_fast}
hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include --offload-device-only -c -o /dev/null \
    -Rpass-analysis=kernel-resource-usage "stateright_amd/csrc/$SRC" 2>&1 |
    awk -v pat="$PAT" '/Function Name:/ {show = ($0 ~ pat); if (show) print ""} show && /remark/ {sub(/.*remark: /, ""); print}'
