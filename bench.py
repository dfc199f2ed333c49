#!/usr/bin/env python3
"""Benchmark: unique states/sec of Stateright's `spawn_bfs` on 2pc N=9 (BASELINE.json), MI355X engine.

One "step" = one complete breadth-first check of TwoPhaseSys{rms: 0..9} (10 340 352 unique /
123 558 402 generated states, 28 levels), spawn -> join, on device-resident buffers (the device
allocator caches the visited set and frontiers across steps; the per-step memset of the visited
set is inside the timed region).

    python bench.py [--gpus N] [--steps K] [--warmup W]

N > 1 runs under torch.distributed.run, one process per GPU, and partitions ONE check over the
GPUs: the visited set and frontier are hash-partitioned by fingerprint owner and
every BFS level does one RCCL all-gather + one all-to-all of successor records over xGMI. The
workload stays 2pc N=9 at every N ("scaling": "strong"); value = unique states of the check /
max-over-ranks time. `--mode replicas` instead runs an independent full check per GPU.

Prints ONE JSON line on rank 0 with `roofline` (dominant kernel = the expand kernel, HIP-event
timed on its own stream inside the engine) and `cpu_baseline` (the CPU restatement of the
reference `spawn_bfs`, oracle/bfs_cli, timed on this host's cores on a bounded sample).
"""
import argparse
import json
import os
import re
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--model", default="2pc", choices=["2pc", "paxos", "increment_lock"],
                    help="workload (the BASELINE metric is 2pc; the others are side measurements)")
    ap.add_argument("--rm-count", type=int, default=9)
    ap.add_argument("--clients", type=int, default=3, help="paxos client_count")
    ap.add_argument("--threads", type=int, default=10, help="increment_lock thread count")
    ap.add_argument("--order", default="fast", choices=["fast", "fifo"])
    ap.add_argument("--cpu-baseline", type=int, default=1, help="time the CPU restatement (rank 0, N=1)")
    ap.add_argument("--cpu-threads", type=int, default=16, help="host threads for the CPU baseline")
    ap.add_argument("--cpu-rm-count", type=int, default=8, help="2pc size of the bounded CPU sample")
    ap.add_argument("--mode", default="partitioned", choices=["partitioned", "replicas", "rccl1"],
                    help="N>1: one check partitioned over the GPUs, or one independent check per GPU; "
                         "rccl1: the partitioned RCCL path on a one-rank communicator (N=1 rehearsal)")
    return ap.parse_args()


def cpu_baseline(args):
    """The oracle's restatement of the multi-threaded reference BFS (oracle/bfs_cli), bounded sample."""
    cli = os.path.join(ROOT, "oracle", "bfs_cli")
    if not os.path.exists(cli):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    threads = max(1, min(args.cpu_threads, os.cpu_count() or 1))
    if args.model == "paxos":
        cmd, what = ["paxos", str(args.clients)], f"paxos C={args.clients}"
    elif args.model == "increment_lock":
        cmd, what = ["increment_lock", str(min(args.threads, 9))], f"increment_lock N={min(args.threads, 9)}"
    else:
        cmd, what = ["2pc", str(args.cpu_rm_count)], f"2pc N={args.cpu_rm_count}"
    def timed(t):
        out = subprocess.run([cli] + cmd + [str(t)], capture_output=True, text=True, timeout=600, check=True).stdout
        m = re.search(r"RESULT state_count=(\d+) unique=(\d+) max_depth=(\d+) threads=(\d+) sec=([\d.e+-]+)", out)
        return int(m[1]), int(m[2]), int(m[4]), float(m[5])

    runs = [timed(threads), timed(1)]  # nproc-like threads, and the reference's default thread_count (src/checker.rs:45)
    sc, uq, th, sec = max(runs, key=lambda r: r[1] / r[3])  # the better of the two is the baseline
    return {
        "value": uq / sec,
        "by_threads": {str(r[2]): r[1] / r[3] for r in runs},
        "unit": "unique states/s",
        "cores": th,
        "kind": "port",
        "sample": f"full {what} check ({uq} unique / {sc} generated states) in {sec:.2f} s "
                  f"on {th} host threads: C++ restatement of src/checker/bfs.rs (job market, sharded "
                  f"visited map, shared state_count atomic); the Rust reference cannot be built here",
    }


# Random 64-bit atomicCAS into a >= 64 MiB table on MI355X, measured by scripts/microbench_random.hip
# (profiles/r01_microbench_random_access.txt): the ceiling of the visited-set claims.
RANDOM_CAS_PEAK = 26.9e9


def pmc_traffic(n, world):
    """Beyond-L2 bytes per expand launch from the committed rocprofv3 PMC passes of this bench
    (scripts/pmc_traffic.sh -> profiles/pmc_traffic.json), or None if not measured for this config."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        if d.get("rm_count") == n and d.get("n_gpus", 1) == world:
            return d["bytes_per_launch"], d.get("atomics_per_launch")
    except (OSError, ValueError, KeyError):
        pass
    return None, None


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl")
    else:
        torch.cuda.set_device(0)
    dev = torch.cuda.current_device()

    import math

    from stateright_amd import IncrementLock, Paxos, TwoPhaseSys
    n = args.rm_count
    if args.model == "paxos":
        make = lambda: Paxos(args.clients)  # noqa: E731
        expect_unique = {1: 265, 2: 16_668, 3: 1_194_428}[args.clients]
        label = f"paxos C={args.clients}"
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
    if partitioned:
        from stateright_amd.distributed import Communicator
        comm = Communicator.from_torch(device=dev) if world > 1 else Communicator(0, 1, Communicator.unique_id(), dev)

    def step(profile=False):
        b = make().checker().capacity_hint(expect_unique).device(dev)
        b = b.comm(comm) if partitioned else b.order(args.order)
        if profile:
            b = b.profile()
        c = b.spawn_bfs().join()
        if c.unique_state_count() != expect_unique:
            raise SystemExit(f"wrong unique count {c.unique_state_count()} != {expect_unique}")
        return c

    for _ in range(args.warmup):
        step()

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    # Timed region of `value`: K full checks without per-launch events (a HIP event pair around
    # every level launch adds a marker packet between the kernels: ~7% of a 2pc N=9 check).
    barrier()
    t0 = time.perf_counter()
    unique = 0
    for _ in range(args.steps):
        c = step()
        unique += c.unique_state_count()
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
    for _ in range(args.steps):
        c = step(profile=True)
        st = c.stats()
        kernel_ms += st["expand_kernel_ms"]
        launches += st["expand_launches"]
        alg_bytes += st["algorithmic_bytes"]
        last = (c, st)
    barrier()
    profiled_elapsed = time.perf_counter() - t1
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        if partitioned:
            unique_total = float(unique)  # every rank reports the global count of the shared check
        else:
            u = torch.tensor([unique], dtype=torch.float64, device="cuda")
            dist.all_reduce(u)
            unique_total = float(u.item())
    else:
        unique_total = float(unique)

    if rank != 0:
        del c
        if comm is not None:
            comm.close()
        if dist is not None:
            dist.destroy_process_group()
        return

    c, st = last
    avg_launch_ms = kernel_ms / max(1, launches)
    if partitioned:
        alg_bytes /= world  # this rank's share of the check's algorithmic bytes
    achieved_gbps = alg_bytes / (kernel_ms * 1e-3) / 1e9 if kernel_ms else 0.0
    traffic, atomics = pmc_traffic(n, world) if args.model == "2pc" and not partitioned else (None, None)
    launch_s = avg_launch_ms * 1e-3
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
            "order": args.order,
            "parallelism": (f"partitioned{world} (RCCL all-to-all per level)" if partitioned else
                            f"replicas{world}" if world > 1 else "1 GPU"),
        },
        "state_count_per_sec": float(c.state_count()) * world * args.steps / elapsed,
        "roofline": {
            "bound": "hbm",
            "kernel": ("expand_route" if partitioned else "expand_fast") +
                      " (expand + fingerprint + visited-set probe/claim + append + properties)",
            "achieved": achieved_gbps,
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": achieved_gbps / HBM_PEAK_GBPS,
            "traffic": traffic,
            # the PMC bytes and memory-side atomics per launch over the event-timed launch duration
            "traffic_gbps": traffic / launch_s / 1e9 if traffic and launch_s else None,
            "atomics_per_s": atomics / launch_s if atomics and launch_s else None,
            "atomics_peak_per_s": RANDOM_CAS_PEAK if atomics else None,
            "avg_launch_ms": avg_launch_ms,
            "launches_per_step": launches / args.steps,
            "algorithmic_bytes_per_step": alg_bytes / args.steps,
            "profiled_ms_per_step": profiled_elapsed / args.steps * 1e3,
        },
        "engine": {k: st[k] for k in ("levels", "table_capacity", "rehashes", "level_loop_sec", "total_sec",
                                      "restarts", "pipelined", "records_routed")},
    }
    if args.cpu_baseline and world == 1:
        try:
            res["cpu_baseline"] = cpu_baseline(args)
        except Exception as e:  # the GPU number stands on its own
            res["cpu_baseline"] = {"error": str(e)}
    print(json.dumps(res))
    if comm is not None:
        comm.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
