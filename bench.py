#!/usr/bin/env python3
"""Benchmark: unique states/sec of Stateright's `spawn_bfs` on 2pc N=9 (BASELINE.json), MI355X engine.

One "step" = one complete breadth-first check of TwoPhaseSys{rms: 0..9} (10 340 352 unique /
123 558 402 generated states, 28 levels), spawn -> join, on device-resident buffers (the device
allocator caches the visited set and frontiers across steps; the per-step memset of the visited
set is inside the timed region).

    python bench.py [--gpus N] [--steps K] [--warmup W]

N > 1: one process per GPU. If WORLD_SIZE is not set, this script starts
`python -m torch.distributed.run --nproc-per-node N ... bench.py ...` as a CHILD process (before
anything touches the GPU) and exits with its status; under the launcher every rank checks
WORLD_SIZE == N. The ranks partition ONE check: the visited set and the frontier
are hash-partitioned by fingerprint owner; after a few replicated head levels, every BFS level is
exchanged DIRECTLY: each rank's expand kernel stores its records into the owners' receive buffers
through IPC-mapped peer pointers and raises a per-level flag there, and each owner's stream waits
for the flags on the device (no collective and no host step per level). SR_DIRECT=0, or a failed
one-off probe of the peer path, falls back to ONE RCCL all-to-all of fixed-capacity buckets per
level (whose headers carry every rank's row). DESIGN.md §6.
The workload stays 2pc N=9 at every N ("scaling": "strong"); value = unique states of the check /
max-over-ranks time. At N > 1 the line also carries `replicas`: the whole node's throughput on
independent full checks (one per GPU and step, weak scaling). `--mode replicas` makes that the
`value` instead.

torch is never imported: the engine library (and with it /opt/rocm's HIP runtime and RCCL, the ones
it was compiled against) is the only GPU runtime in the process; ranks bootstrap RCCL from the
launcher's environment (stateright_amd.distributed.Communicator.from_env) and the timing barrier /
max-over-ranks are the engine's own (sr_dist_barrier, sr_dist_allreduce_f64).

Prints ONE JSON line on rank 0 with `roofline` (dominant kernel = the expand kernel, HIP-event
timed on the engine's stream) and, at N=1, `cpu_baseline` (the CPU restatement of the reference
`spawn_bfs`, oracle/bfs_cli, on the same 2pc N=9 check, host threads and 1 thread).
"""
import argparse
import contextlib
import ctypes
import json
import os
import re
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# Uniform random-access rates into a 256 MiB table (scripts/microbench_random.hip,
# profiles/r01_microbench_random_access.txt): reported beside the kernel's probe and claim rates
# for context only. They are NOT ceilings of the kernel (its probes hit L2 29% of the time and its
# linear-probe steps stay in a line), so they enter no fraction; the memory-side bounds are the
# PMC-measured request ceilings of profiles/pmc_ceiling.json.
UNIFORM_LOAD_RATE = 55.6e9
UNIFORM_CAS_RATE = 26.7e9
BIG_LEVEL_MS = 0.1  # levels whose expand launch takes >= 100 us count as "big"



def _proc_start(pid):
    """Start time of process `pid` in clock ticks since boot (/proc/<pid>/stat field 22), or 0."""
    try:
        with open(f"/proc/{pid}/stat") as f:
            return int(f.read().rsplit(")", 1)[1].split()[19])
    except (OSError, IndexError, ValueError):
        return 0

def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="2pc", choices=["2pc", "paxos", "increment_lock", "single_copy"],
                    help="workload (the BASELINE metric is 2pc; the others are side measurements)")
    ap.add_argument("--rm-count", type=int, default=9)
    ap.add_argument("--clients", type=int, default=3, help="paxos / single_copy client_count")
    ap.add_argument("--threads", type=int, default=10, help="increment_lock thread count")
    ap.add_argument("--order", default="fast", choices=["fast", "fifo"])
    ap.add_argument("--cpu-baseline", type=int, default=1, help="time the CPU restatement (rank 0, N=1)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="host threads for the CPU baseline (0 = usable CPUs)")
    ap.add_argument("--no-hint-steps", type=int, default=10,
                    help="checks timed WITHOUT capacity_hint (reported as `no_hint`; 0 = skip)")
    ap.add_argument("--config4-steps", type=int, default=3,
                    help="also time BASELINE configs[3] (2pc N=11, partitioned over the N GPUs; one GPU at N=1) "
                         "for this many checks after one warmup (0 = skip); reported as `config4`, not `value`")
    ap.add_argument("--comm", default="rccl", choices=["rccl", "shm"],
                    help="N>1 host-side transport: RCCL (one process per GPU), or a shared-memory segment "
                         "(a rehearsal of the multi-process path with every rank on ONE GPU, where RCCL refuses "
                         "two ranks on one device; its timings are not the node's)")
    ap.add_argument("--dry-run", action="store_true",
                    help="every rank prints its launch plan as JSON and exits before any GPU call")
    ap.add_argument("--mode", default="partitioned", choices=["partitioned", "replicas", "rccl1"],
                    help="N>1: one check partitioned over the GPUs, or one independent check per GPU; "
                         "rccl1: the partitioned RCCL path on a one-rank communicator (N=1 rehearsal)")
    return ap.parse_args()


@contextlib.contextmanager
def stdout_to_stderr():
    """fd 1 -> fd 2 for the duration (RCCL prints its init banner to stdout with C stdio; the
    bench's stdout must carry only the JSON line)."""
    sys.stdout.flush()
    libc = ctypes.CDLL(None)
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        yield
    finally:
        libc.fflush(None)
        os.dup2(saved, 1)
        os.close(saved)


def launch_ranks(args):
    """Starts one process per GPU under torch.distributed.run as a child and returns its status."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.run(cmd, env=env).returncode


def cpu_info():
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count() or 1
    try:  # a cgroup CPU quota (the GPU box gives a share of the machine) bounds it further
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            usable = max(1, min(usable, int(int(quota) / int(period))))
    except (OSError, ValueError):
        pass
    return model, os.cpu_count() or 1, usable


def cpu_baseline(args, n):
    """The oracle's restatement of the multi-threaded reference BFS (oracle/bfs_cli) on the SAME
    check as the GPU line, at the usable host threads and at 1 thread (the reference's default
    thread_count, src/checker.rs:45)."""
    cli = os.path.join(ROOT, "oracle", "bfs_cli")
    if not os.path.exists(cli):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    model, nproc, usable = cpu_info()
    threads = args.cpu_threads or usable
    if args.model == "paxos":
        cmd, what = ["paxos", str(args.clients)], f"paxos C={args.clients}"
    elif args.model == "single_copy":
        cmd, what = ["single_copy", str(args.clients)], f"single-copy register C={args.clients}"
    elif args.model == "increment_lock":
        cmd, what = ["increment_lock", str(min(args.threads, 9))], f"increment_lock N={min(args.threads, 9)}"
    else:
        cmd, what = ["2pc", str(n)], f"2pc N={n}"

    def timed(t):
        out = subprocess.run([cli] + cmd + [str(t)], capture_output=True, text=True, timeout=900, check=True).stdout
        m = re.search(r"RESULT state_count=(\d+) unique=(\d+) max_depth=(\d+) threads=(\d+) sec=([\d.e+-]+)", out)
        done = next((ln for ln in out.splitlines() if ln.startswith("Done. ")), None)
        return {"state_count": int(m[1]), "unique": int(m[2]), "threads": int(m[4]), "sec": float(m[5]), "done": done}

    runs = [timed(threads)] + ([timed(1)] if threads != 1 else [])
    best = max(runs, key=lambda r: r["unique"] / r["sec"])
    return {
        "value": best["unique"] / best["sec"],
        "unit": "unique states/s",
        "cores": best["threads"],
        "kind": "port",
        "by_threads": {str(r["threads"]): r["unique"] / r["sec"] for r in runs},
        "done_lines": {str(r["threads"]): r["done"] for r in runs},
        "nproc": nproc,
        "usable_cpus": usable,
        "cpu_model": model,
        "sample": f"full {what} check ({best['unique']} unique / {best['state_count']} generated states) in "
                  f"{best['sec']:.2f} s on {best['threads']} host threads (also timed: "
                  f"{', '.join(str(r['threads']) for r in runs)} threads): the C++ restatement of "
                  f"src/checker/bfs.rs (job market, sharded visited map, shared state_count atomic); the Rust "
                  f"reference cannot be built here (no cargo/rustc)",
    }


def pmc_files(label, world):
    """The committed rocprofv3 PMC measurements of this configuration's expand kernel and the
    measured memory-side request ceilings (scripts/gpu_roofline.sh -> profiles/pmc_traffic.json,
    profiles/pmc_ceiling.json), or (None, None, reason): both files must carry the source digest of
    the engine being benchmarked (stateright_amd.build.source_digest), so a measurement of other
    sources is never reported."""
    from stateright_amd.build import source_digest
    if world != 1:
        return None, None, "PMC files are single-GPU measurements"
    digest = source_digest()
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_traffic.json")) as f:
            traffic = json.load(f)
        with open(os.path.join(ROOT, "profiles", "pmc_ceiling.json")) as f:
            ceiling = json.load(f)
    except (OSError, ValueError):
        return None, None, "no PMC files"
    if traffic.get("source_digest") != digest or ceiling.get("source_digest") != digest:
        return None, None, f"PMC files measured on other sources ({traffic.get('source_digest')} != {digest})"
    cfg = traffic.get("configs", {}).get(label)
    if not cfg:
        return None, None, f"no PMC measurement of {label}"
    return cfg, ceiling, traffic.get("source_digest")


def exchange_label(st):
    """How a partitioned check's levels exchanged their records (sr_stats.pipelined)."""
    return {2: "direct exchange: peer stores + device flags per level",
            1: "RCCL all-to-all per level", 0: "synchronous: all-gather + exchange per level"}.get(st["pipelined"], "?")


def measure_config4(args, world, comm, dev, barrier):
    """BASELINE.json configs[3]: 2pc N=11 (366 993 408 unique states, 34 levels) partitioned over
    the `world` GPUs (one process each; the direct exchange, or RCCL all-to-all with SR_DIRECT=0),
    or on the one GPU at N=1."""
    from stateright_amd import TwoPhaseSys
    n = 11
    want = 6 ** n + 4 ** n + 2 ** n

    def check():
        b = TwoPhaseSys(n).checker().capacity_hint(want).device(dev)
        b = b.comm(comm).defer_paths() if world > 1 else b.order("fast")
        c = b.spawn_bfs().join()
        if c.unique_state_count() != want:
            raise SystemExit(f"config4: wrong unique count {c.unique_state_count()} != {want}")
        return c

    check()  # warmup: allocations
    barrier()
    t0 = time.perf_counter()
    c = None
    for _ in range(args.config4_steps):
        c = None
        c = check()
    barrier()
    el = time.perf_counter() - t0
    if world > 1:
        el = comm.allreduce([el], "max")[0]
    st = c.stats()
    return {"workload": f"2pc N={n} spawn_bfs, full check per step ({want} unique states; BASELINE configs[3])",
            "parallelism": f"partitioned{world} ({exchange_label(st)})" if world > 1 else "1 GPU",
            "n_gpus": world, "steps": args.config4_steps, "ms_per_step": el / args.config4_steps * 1e3,
            "value": want * args.config4_steps / el, "unit": "unique states/s",
            "restarts": st["restarts"], "head_levels": st["head_levels"], "records_routed": st["records_routed"]}


def measure_replicas(args, world, comm, dev, make, expect_unique, label, barrier):
    """N > 1, beside the partitioned `value`: the whole node's throughput on INDEPENDENT checks of
    the same workload (every rank runs one full single-GPU check per step on its own GPU, no
    collective inside a check: weak scaling)."""
    def check():
        c = make().checker().capacity_hint(expect_unique).device(dev).order("fast").spawn_bfs().join()
        if c.unique_state_count() != expect_unique:
            raise SystemExit(f"replicas: wrong unique count {c.unique_state_count()} != {expect_unique}")

    check()  # warmup
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        check()
    barrier()
    el = comm.allreduce([time.perf_counter() - t0], "max")[0]
    return {"workload": f"{label} spawn_bfs, one independent full check per GPU and step",
            "parallelism": f"replicas{world} (no collective inside a check)", "scaling": "weak",
            "n_gpus": world, "steps": args.steps, "ms_per_step": el / args.steps * 1e3,
            "value": float(expect_unique) * world * args.steps / el, "unit": "unique states/s"}


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"rank {rank}: WORLD_SIZE={world} but --gpus {args.gpus}")
    if args.dry_run:
        plan = json.dumps({"dry_run": True, "rank": rank, "world_size": world, "local_rank": local_rank,
                           "device": local_rank if world > 1 else 0, "mode": args.mode,
                           "master": f"{os.environ.get('MASTER_ADDR')}:{os.environ.get('MASTER_PORT')}"})
        sys.stdout.flush()
        os.write(1, (plan + "\n").encode())  # one write: the ranks share the launcher's stdout pipe
        return

    import math

    from stateright_amd import IncrementLock, Paxos, SingleCopyRegister, TwoPhaseSys
    from stateright_amd import _native as N
    lib = N.load()
    # one GPU per rank: LOCAL_RANK when every rank sees the node's GPUs; a launcher that restricts
    # each rank's visible devices leaves fewer (then the rank's own GPU is visible device 0)
    ndev = lib.sr_device_count()
    if ndev < 1:
        raise SystemExit(f"rank {rank}: no GPU visible ({N.last_error()})")
    dev = (local_rank % ndev) if world > 1 else 0
    versions = N.runtime_versions()
    hip_rt, hip_cc = versions["hip"]
    rccl_rt, rccl_cc = versions["rccl"]
    if rccl_rt != rccl_cc or (hip_rt or 0) // 100000 != (hip_cc or 0) // 100000:
        raise SystemExit(f"runtime skew: engine built against HIP {hip_cc} / RCCL {rccl_cc}, "
                         f"running HIP {hip_rt} / RCCL {rccl_rt} ({N.loaded_runtime_paths()})")

    n = args.rm_count
    if args.model == "paxos":
        make = lambda: Paxos(args.clients)  # noqa: E731
        expect_unique = {1: 265, 2: 16_668, 3: 1_194_428, 4: 2_372_188, 5: 4_711_569, 6: 9_357_525}[args.clients]
        label = f"paxos C={args.clients}"
    elif args.model == "single_copy":  # the reference's bench.sh: `single-copy-register check 4`
        make = lambda: SingleCopyRegister(args.clients, 1)  # noqa: E731
        expect_unique = {1: 5, 2: 93, 3: 4_243, 4: 400_233}[args.clients]
        label = f"single-copy register C={args.clients}"
    elif args.model == "increment_lock":
        t = args.threads
        make = lambda: IncrementLock(t)  # noqa: E731
        expect_unique = 1 + 4 * sum(math.factorial(t) // math.factorial(t - k) for k in range(1, t + 1))
        label = f"increment_lock N={t}"
    else:
        make = lambda: TwoPhaseSys(n)  # noqa: E731
        expect_unique = 6 ** n + 4 ** n + 2 ** n
        label = f"2pc N={n}"
    partitioned = (world > 1 and args.mode == "partitioned") or args.mode == "rccl1"
    comm = None
    if world > 1 or args.mode == "rccl1":
        from stateright_amd.distributed import Communicator
        with stdout_to_stderr():
            if args.comm == "shm":
                # every rank names the same segment (the launcher's port, pid and start time: unique
                # per launch); ranks share a GPU when the node has fewer GPUs than ranks
                name = f"/sr_bench_{os.environ.get('MASTER_PORT', '0')}_{os.getppid()}_{_proc_start(os.getppid())}"
                comm = Communicator.shm(rank, world, name, device=dev, slot_bytes=256 << 20,
                                        devices_distinct=ndev >= world)
            # under a launcher (RANK set) every rank bootstraps from its environment, also at N=1
            else:
                comm = (Communicator.from_env(device=dev) if "RANK" in os.environ
                        else Communicator(0, 1, Communicator.unique_id(), dev))

    def step(profile=False, counters=False, hint=True):
        b = make().checker().device(dev)
        if hint:  # the headline is pre-sized; `no_hint` times the path users get (no such option
            b = b.capacity_hint(expect_unique)  # in the reference, src/checker.rs:35-51)
        if counters:
            b = b.counters()
        # the reference's join reconstructs no paths (discoveries() does, bfs.rs:289-298): the
        # partitioned check skips gathering them at join as well
        b = b.comm(comm).defer_paths() if partitioned else b.order(args.order)
        if profile:
            b = b.profile()
        c = b.spawn_bfs().join()
        if c.unique_state_count() != expect_unique:
            raise SystemExit(f"wrong unique count {c.unique_state_count()} != {expect_unique}")
        return c

    # A finished checker holds its visited set and arena until it is freed: drop the previous one
    # before the next check allocates (increment_lock N=12 needs ~200 GB of the 288).
    for _ in range(args.warmup):
        step()

    def barrier():
        if comm is not None and world > 1:
            comm.barrier()  # device sync of this rank + collective
        elif lib.sr_device_synchronize(dev) != 0:
            raise SystemExit(N.last_error())

    # Timed region of `value`: K full checks without per-launch events (a HIP event pair around
    # every level launch adds a marker packet between the kernels: ~7% of a 2pc N=9 check).
    barrier()
    t0 = time.perf_counter()
    unique = 0
    c = None
    for _ in range(args.steps):
        c = None
        c = step()
        unique += c.unique_state_count()
    # the last checker is freed inside the timed region too: a freed checker's visited set is
    # cleared on the device behind it (the next check takes it clean), so every step pays its clear
    c = None
    barrier()
    elapsed = time.perf_counter() - t0

    # Roofline pass: the same K checks again with HIP events around every expand launch, on the
    # engine's own stream; achieved bytes / summed event time of the dominant kernel.
    kernel_ms = 0.0
    launches = 0
    alg_bytes = 0
    last = None
    barrier()
    t1 = time.perf_counter()
    c = None
    for _ in range(args.steps):
        c = last = None
        c = step(profile=True)
        st = c.stats()
        kernel_ms += st["expand_kernel_ms"]
        launches += st["expand_launches"]
        alg_bytes += st["algorithmic_bytes"]
        last = (c, st)
    barrier()
    profiled_elapsed = time.perf_counter() - t1
    # Counter pass (untimed): visited-set probes and CAS claims per check, from a counting variant
    # of the expand kernel; the rates divide them by the event-timed kernel time of the pass above.
    c, st = last
    last = None
    prof = c.launch_profile() if not partitioned else []
    final_state_count = c.state_count()
    c = None
    probes = cas = 0
    per_launch = []
    for _ in range(args.steps):
        cc = step(counters=True)
        stc = cc.stats()
        probes += stc["probes"]
        cas += stc["cas"]
        per_launch = cc.launch_counters() if not partitioned else []
        cc = None
    if world > 1:
        elapsed = comm.allreduce([elapsed], "max")[0]
    unique_total = float(unique) if partitioned or world == 1 else float(unique) * world

    # The path users get: the same checks without capacity_hint (the visited set and the arena grow
    # during the check, as the reference's DashMap does). Not `value`: reported beside it.
    no_hint = None
    if args.no_hint_steps > 0:
        step(hint=False)  # warmup
        barrier()
        t2 = time.perf_counter()
        c = None
        for _ in range(args.no_hint_steps):
            c = None
            c = step(hint=False)
        stn = c.stats()
        c = None
        barrier()
        el_nh = time.perf_counter() - t2
        if world > 1:
            el_nh = comm.allreduce([el_nh], "max")[0]
        nh_total = expect_unique * args.no_hint_steps * (1 if partitioned or world == 1 else world)
        no_hint = {"steps": args.no_hint_steps, "ms_per_step": el_nh / args.no_hint_steps * 1e3,
                   "value": nh_total / el_nh, "unit": "unique states/s",
                   "rehashes": stn["rehashes"], "table_capacity": stn["table_capacity"], "restarts": stn["restarts"]}

    config4 = None
    if args.config4_steps > 0 and args.model == "2pc":
        config4 = measure_config4(args, world, comm, dev, barrier)
    replicas = None
    # (SR_BENCH_REPLICAS=1 runs it at N=1 in --mode rccl1 too: the rehearsal of this code path)
    if partitioned and (world > 1 or os.environ.get("SR_BENCH_REPLICAS") == "1"):
        replicas = measure_replicas(args, world, comm, dev, make, expect_unique, label, barrier)

    if rank != 0:
        comm.close()
        return

    avg_launch_ms = kernel_ms / max(1, launches)
    if partitioned:
        alg_bytes /= world  # this rank's share of the check's algorithmic bytes
    kernel_s = kernel_ms * 1e-3
    achieved_gbps = alg_bytes / kernel_s / 1e9 if kernel_ms else 0.0
    pmc, ceiling, pmc_note = pmc_files(label, world) if not partitioned else (None, None, "partitioned run")
    launch_s = avg_launch_ms * 1e-3
    probe_rate = probes / kernel_s if kernel_s and probes else None
    cas_rate = cas / kernel_s if kernel_s and cas else None
    # Fractions of bounds the kernel cannot exceed: algorithmic bytes against HBM's 8 TB/s, and
    # (when a PMC measurement of these sources exists) its memory-side read / write / atomic
    # requests per second against the largest rates the random-access microbenchmark reached.
    fracs = {"hbm_bytes": achieved_gbps / HBM_PEAK_GBPS}
    ea = None
    if pmc and launch_s:
        ea = {"read_req_per_s": pmc["ea_read_req_per_launch"] / launch_s,
              "write_req_per_s": pmc["ea_write_req_per_launch"] / launch_s,
              "atomic_req_per_s": pmc["ea_atomic_req_per_launch"] / launch_s,
              "read_req_peak": ceiling["ea_read_req_per_s"], "write_req_peak": ceiling["ea_write_req_per_s"],
              "atomic_req_peak": ceiling["ea_atomic_req_per_s"]}
        fracs["ea_read_requests"] = ea["read_req_per_s"] / ceiling["ea_read_req_per_s"]
        fracs["ea_write_requests"] = ea["write_req_per_s"] / ceiling["ea_write_req_per_s"]
        fracs["ea_atomic_requests"] = ea["atomic_req_per_s"] / ceiling["ea_atomic_req_per_s"]
        fracs["hbm_traffic"] = pmc["bytes_per_launch"] / launch_s / 1e9 / HBM_PEAK_GBPS
    traffic = pmc["bytes_per_launch"] if pmc else None
    # The big levels alone (launches >= BIG_LEVEL_MS of the profiled check): probes and CAS claims
    # per second of their event time (context: the whole-check rates are diluted by small levels).
    big_rate = None
    if prof and len(per_launch) == len(prof):
        bi = [i for i, (ms, _) in enumerate(prof) if ms >= BIG_LEVEL_MS]
        bt = sum(prof[i][0] for i in bi) * 1e-3
        bp, bc = sum(per_launch[i][0] for i in bi), sum(per_launch[i][1] for i in bi)
        if bt > 0 and bp:
            big_rate = {"launches": len(bi), "probe_rate": bp / bt, "cas_rate": bc / bt}
    # Per-level split of the last profiled check: big levels, small levels, and the span between
    # launches (level boundaries: dispatch, ramp/drain, host planning).
    big = sum(ms for ms, _ in prof if ms >= BIG_LEVEL_MS)
    small = sum(ms for ms, _ in prof if ms < BIG_LEVEL_MS)
    span_ms = st["level_loop_sec"] * 1e3
    res = {
        "metric": "unique states/sec (whole node) + HBM GB/s, 2pc N=9 at 1/2/4/8 MI355X",
        "value": unique_total / elapsed,
        "unit": "unique states/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong" if (world == 1 or partitioned) else "weak",
        "vs_baseline": None,
        "dtype": "u64",
        "data": f"synthetic: the {args.model} model's own state space (no dataset)",
        "config": {
            "workload": f"{label} spawn_bfs, full check per step ({expect_unique} unique states)",
            "model": args.model,
            "rm_count": n if args.model == "2pc" else None,
            "order": "fast" if partitioned else args.order,
            "parallelism": (f"partitioned{world} ({exchange_label(st)})" if partitioned else
                            f"replicas{world}" if world > 1 else "1 GPU"),
            "world_size": world,
            "comm": comm.kind() if comm is not None else None,
            "rccl_nranks": comm.nranks() if comm is not None else None,
        },
        "state_count_per_sec": float(final_state_count) * (1 if partitioned else world) * args.steps / elapsed,
        "roofline": {
            # HBM-side: random visited-set probes and claims (8-byte accesses that each move a
            # memory line) and streamed frontiers. `limiter` names the largest fraction of a bound
            # the kernel cannot exceed.
            "bound": "hbm",
            "limiter": max(fracs, key=fracs.get),
            "fractions": fracs,
            "kernel": ("expand_route" if partitioned else "expand_fast") +
                      " (expand + fingerprint + visited-set probe/claim + append + properties)",
            "achieved": achieved_gbps,
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": achieved_gbps / HBM_PEAK_GBPS,
            "traffic": traffic,
            "traffic_gbps": traffic / launch_s / 1e9 if traffic and launch_s else None,
            "memory_side_requests": ea,
            "pmc": pmc_note,
            # context: visited-set probes and claims per second of kernel time (device counters)
            # beside the uniform random-access rates of one 256 MiB table
            "probe_rate": probe_rate,
            "cas_rate": cas_rate,
            "uniform_load_rate": UNIFORM_LOAD_RATE,
            "uniform_cas_rate": UNIFORM_CAS_RATE,
            "probes_per_step": probes / args.steps,
            "big_levels": big_rate,
            "avg_launch_ms": avg_launch_ms,
            "launches_per_step": launches / args.steps,
            "algorithmic_bytes_per_step": alg_bytes / args.steps,
            "profiled_ms_per_step": profiled_elapsed / args.steps * 1e3,
        },
        "levels": {
            "span_ms": span_ms,
            "big_levels_ms": big,
            "big_levels": sum(1 for ms, _ in prof if ms >= BIG_LEVEL_MS),
            "small_levels_ms": small,
            "small_levels": sum(1 for ms, _ in prof if ms < BIG_LEVEL_MS),
            "gaps_ms": max(0.0, span_ms - big - small) if prof else None,
            "kernel_us": [round(ms * 1e3, 1) for ms, _ in prof],
            "frontier": [fr for _, fr in prof],
            # visited-set loads and CAS claims of each launch (counting pass): DESIGN.md §3's
            # attribution of the level times
            "probes": [int(p) for p, _ in per_launch] if len(per_launch) == len(prof) else None,
            "cas": [int(c) for _, c in per_launch] if len(per_launch) == len(prof) else None,
        } if prof else None,
        "engine": {k: st[k] for k in ("levels", "table_capacity", "rehashes", "level_loop_sec", "total_sec",
                                      "restarts", "pipelined", "records_routed", "head_levels")},
        "runtime": {"hip": versions["hip"], "rccl": versions["rccl"], "libs": N.loaded_runtime_paths(),
                    "lib_digest": N.build_digest(), "source_digest": __import__("stateright_amd.build").build.source_digest()},
    }
    if no_hint is not None:
        no_hint["vs_value"] = no_hint["value"] / res["value"]
        res["no_hint"] = no_hint
    if config4 is not None:
        res["config4"] = config4
    if replicas is not None:
        res["replicas"] = replicas
    if args.cpu_baseline and world == 1:
        try:
            res["cpu_baseline"] = cpu_baseline(args, n)
        except Exception as e:  # the GPU number stands on its own
            res["cpu_baseline"] = {"error": str(e)}
    print(json.dumps(res), flush=True)
    if comm is not None:
        comm.close()


if __name__ == "__main__":
    main()
