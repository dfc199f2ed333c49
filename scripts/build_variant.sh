#!/bin/bash
# An A/B variant of the engine library: the named registry units recompiled with extra -D defines,
# linked with the in-tree objects of every other unit into gpurun_ab/lib_<name>.so (for
# scripts/gpu_lib_ab.sh / gpu_quick_ab.sh; the in-tree library is untouched).
#   scripts/build_variant.sh <name> "<unit.hip> ..." -DFOO=1 ...
set -e
cd "$(dirname "$0")/.."
NAME=${1:?name}; UNITS=${2:?units}; shift 2
python -c "import stateright_amd.build as b; b.build()"
OBJ=stateright_amd/build
VO=gpurun_ab/obj_$NAME
rm -rf "$VO"  # no stale object of an earlier, interrupted run can be linked in
mkdir -p "$VO"
objs=()
pids=()
for o in $OBJ/*.o; do
    u=$(basename "$o" .o).hip
    if [[ " $UNITS " == *" $u "* ]]; then
        hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -I include "$@" -c -o "$VO/${u%.hip}.o" "stateright_amd/csrc/$u" &
        pids+=($!)
        objs+=("$VO/${u%.hip}.o")
    else
        objs+=("$o")
    fi
done
for pid in "${pids[@]}"; do  # a bare `wait` returns 0 even when a compile failed
    wait "$pid" || { echo "build_variant: a compile failed" >&2; exit 1; }
done
hipcc --offload-arch=gfx950 -shared -fPIC -o "gpurun_ab/lib_$NAME.so" "${objs[@]}" -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -rf "$VO"
echo "gpurun_ab/lib_$NAME.so"
