"""Builds the in-tree HIP engine library for gfx950 (no JIT cache: the .so travels with the repo),
and the example GpuModel plugin (examples/plugins), which instantiates the same engine headers."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = os.path.join(HERE, "csrc", "engine.hip")
CSRC = [os.path.join(HERE, "csrc", f) for f in ("engine.hip", "engine.hpp", "kernels.hpp", "kernels_dist.hpp",
                                                 "dist.hpp", "models.hpp", "device.hpp", "paxos.hpp", "dgraph.hpp",
                                                 "actor.hpp")]
HEADERS = [os.path.join(ROOT, "include", f) for f in ("stateright_gpu.h", "stateright_gpu_model.hpp")]
OUT = os.path.join(HERE, "libstateright_gpu.so")
PLUGINS = {"sliding_puzzle": os.path.join(ROOT, "examples", "plugins", "sliding_puzzle.hip")}
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")


def plugin_path(name):
    return os.path.join(ROOT, "examples", "plugins", f"lib{name}.so")


def _hipcc(src, out, deps, force, verbose):
    if not force and os.path.exists(out) and all(os.path.getmtime(out) >= os.path.getmtime(d) for d in deps):
        return out
    cmd = ["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wall",
           "-I", os.path.join(ROOT, "include"), "-o", out + ".tmp", src,
           "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    os.replace(out + ".tmp", out)
    return out


# The cross-process check of the direct exchange's IPC path (run by tests/test_gpu_partitioned.py):
# an executable built from the same engine headers.
IPC_SELFTEST_SRC = os.path.join(ROOT, "scripts", "ipc_selftest.hip")
IPC_SELFTEST = os.path.join(ROOT, "scripts", "ipc_selftest")


def _hipcc_exe(src, out, deps, force, verbose):
    if not force and os.path.exists(out) and all(os.path.getmtime(out) >= os.path.getmtime(d) for d in deps):
        return out
    cmd = ["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-I", os.path.join(ROOT, "include"),
           "-o", out + ".tmp", src, "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    os.replace(out + ".tmp", out)
    return out


def build(force=False, verbose=False, plugins=True):
    _hipcc(SRC, OUT, CSRC + HEADERS, force, verbose)
    if plugins:
        for name, src in PLUGINS.items():
            _hipcc(src, plugin_path(name), CSRC + HEADERS + [src], force, verbose)
        _hipcc_exe(IPC_SELFTEST_SRC, IPC_SELFTEST, CSRC + HEADERS + [IPC_SELFTEST_SRC], force, verbose)
    return OUT


if __name__ == "__main__":
    print(build(force=True, verbose=True))


def source_digest():
    """sha256 (16 hex digits) of the engine's sources (CSRC + HEADERS): measurement files under
    profiles/ are stamped with it, and bench.py ignores a file measured on other sources."""
    import hashlib
    h = hashlib.sha256()
    for path in sorted(CSRC + HEADERS):
        with open(path, "rb") as f:
            h.update(os.path.basename(path).encode() + b"\0" + f.read())
    return h.hexdigest()[:16]
