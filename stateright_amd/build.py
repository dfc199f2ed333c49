"""Builds the in-tree HIP engine library for gfx950 (no JIT cache: the .so travels with the repo),
and the example GpuModel plugin (examples/plugins), which instantiates the same engine headers.

The library is several translation units compiled in parallel: engine.hip (the C ABI) and one
reg_<family>.hip per family of registered models (csrc/registry.hpp), each instantiating the
engine's kernels for its models. engine.hip is compiled with the source digest (`source_digest`)
as SR_BUILD_DIGEST, which `sr_build_digest()` returns and `_native.load()` checks."""
import concurrent.futures
import hashlib
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CDIR = os.path.join(HERE, "csrc")
SRC = os.path.join(CDIR, "engine.hip")
UNITS = ["engine.hip", "reg_basic.hip", "reg_two_phase.hip", "reg_increment.hip", "reg_increment_lock.hip",
         "reg_paxos.hip", "reg_paxos_wide.hip", "reg_ping_pong.hip", "reg_registers.hip"]
CSRC = [os.path.join(CDIR, f) for f in UNITS + ["registry.hpp", "engine.hpp", "kernels.hpp", "kernels_dist.hpp",
                                                "dist.hpp", "dist_host.hpp", "models.hpp", "device.hpp", "paxos.hpp", "dgraph.hpp",
                                                "actor.hpp"]]
HEADERS = [os.path.join(ROOT, "include", f) for f in ("stateright_gpu.h", "stateright_gpu_model.hpp")]
OUT = os.path.join(HERE, "libstateright_gpu.so")
OBJDIR = os.path.join(HERE, "build")
PLUGINS = {"sliding_puzzle": os.path.join(ROOT, "examples", "plugins", "sliding_puzzle.hip")}
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
FLAGS = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall", "-I", os.path.join(ROOT, "include")]
LINK = ["-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]


def source_digest():
    """sha256 (16 hex digits) of the engine's sources (CSRC + HEADERS): compiled into the library
    (sr_build_digest), and measurement files under profiles/ are stamped with it (bench.py ignores
    a file measured on other sources)."""
    return source_digest_at(ROOT)


def source_digest_at(root):
    """source_digest of the copy of the sources under another repository root."""
    h = hashlib.sha256()
    for path in sorted(CSRC + HEADERS):
        with open(os.path.join(root, os.path.relpath(path, ROOT)), "rb") as f:
            h.update(os.path.basename(path).encode() + b"\0" + f.read())
    return h.hexdigest()[:16]


def plugin_path(name):
    return os.path.join(ROOT, "examples", "plugins", f"lib{name}.so")


def _fresh(out, deps):
    return os.path.exists(out) and all(os.path.getmtime(out) >= os.path.getmtime(d) for d in deps)


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)


def _hipcc(src, out, deps, force, verbose):
    if not force and _fresh(out, deps):
        return out
    _run(["hipcc"] + FLAGS + ["-shared", "-o", out + ".tmp", src] + LINK, verbose)
    os.replace(out + ".tmp", out)
    return out


# The cross-process check of the direct exchange's IPC path (run by tests/test_gpu_partitioned.py):
# an executable built from the same engine headers.
IPC_SELFTEST_SRC = os.path.join(ROOT, "scripts", "ipc_selftest.hip")
IPC_SELFTEST = os.path.join(ROOT, "scripts", "ipc_selftest")


def _hipcc_exe(src, out, deps, force, verbose):
    if not force and _fresh(out, deps):
        return out
    _run(["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-I", os.path.join(ROOT, "include"),
          "-o", out + ".tmp", src] + LINK, verbose)
    os.replace(out + ".tmp", out)
    return out


def _library(force, verbose, pool):
    """The engine library: every unit to an object (in parallel), then one link."""
    deps = CSRC + HEADERS
    if not force and _fresh(OUT, deps):
        return []
    os.makedirs(OBJDIR, exist_ok=True)
    digest = source_digest()

    def compile_unit(unit):
        obj = os.path.join(OBJDIR, unit.replace(".hip", ".o"))
        extra = [f'-DSR_BUILD_DIGEST="{digest}"'] if unit == "engine.hip" else []
        _run(["hipcc"] + FLAGS + extra + ["-c", "-o", obj + ".tmp", os.path.join(CDIR, unit)], verbose)
        os.replace(obj + ".tmp", obj)
        return obj

    def link(futs):
        objs = [f.result() for f in futs]
        _run(["hipcc", f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", OUT + ".tmp"] + objs + LINK, verbose)
        os.replace(OUT + ".tmp", OUT)
        return OUT

    # the largest units first, so the slowest compiles start first
    order = sorted(UNITS, key=lambda u: 0 if u.startswith("reg_paxos") or u == "reg_registers.hip" else 1)
    return [pool.submit(link, [pool.submit(compile_unit, u) for u in order])]


def build(force=False, verbose=False, plugins=True):
    workers = max(2, min(len(UNITS) + 3, (os.cpu_count() or 4)))
    with concurrent.futures.ThreadPoolExecutor(max_workers=workers + 1) as pool:
        futs = _library(force, verbose, pool)
        if plugins:
            for name, src in PLUGINS.items():
                futs.append(pool.submit(_hipcc, src, plugin_path(name), CSRC + HEADERS + [src], force, verbose))
            futs.append(pool.submit(_hipcc_exe, IPC_SELFTEST_SRC, IPC_SELFTEST, CSRC + HEADERS + [IPC_SELFTEST_SRC],
                                    force, verbose))
        for f in futs:
            f.result()
    return OUT


if __name__ == "__main__":
    print(build(force=True, verbose=True))
