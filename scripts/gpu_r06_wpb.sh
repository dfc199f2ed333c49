#!/bin/bash
# Round 6: 8 waves per workgroup for narrow states (gpurun_ab/lib_wpb8.so, -DSR_NARROW_WPB=8: the LDS
# filter is shared by 512 parents) at the one-residency grid, with the default and a 2^11-entry filter.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_libs_ab.sh r06wpb/n9 3 new wpb8 -- --steps 20 || exit 1
SR_FILTER_LOG2=10 bash scripts/gpu_libs_ab.sh r06wpb/n9f 2 wpb8 -- --steps 20 || exit 1
echo "wpb ok"
