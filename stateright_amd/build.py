"""Builds the in-tree HIP engine library for gfx950 (no JIT cache: the .so travels with the repo)."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "csrc", "engine.hip")
DEPS = [os.path.join(HERE, "csrc", f) for f in ("engine.hip", "kernels.hpp", "kernels_dist.hpp", "dist.hpp",
                                                "models.hpp", "device.hpp", "paxos.hpp", "dgraph.hpp")] + [
    os.path.join(os.path.dirname(HERE), "include", "stateright_gpu.h")]
OUT = os.path.join(HERE, "libstateright_gpu.so")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")


def build(force=False, verbose=False):
    if not force and os.path.exists(OUT) and all(os.path.getmtime(OUT) >= os.path.getmtime(d) for d in DEPS):
        return OUT
    cmd = ["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wall",
           "-o", OUT + ".tmp", SRC, "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force=True, verbose=True))
