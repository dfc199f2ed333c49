#!/bin/bash
# Diagnostic build of the engine with expand_fast's per-workgroup timeline (SR_TIMELINE=1):
# stateright_amd/libstateright_gpu_timeline.so, loaded by scripts/timeline.py through SR_LIB_PATH.
set -e
cd "$(dirname "$0")/.."
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wall -DSR_TIMELINE=1 -DSR_ONE_TU=1 -I include \
    -o stateright_amd/libstateright_gpu_timeline.so stateright_amd/csrc/engine.hip \
    -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
