#!/usr/bin/env python3
"""Per-level decomposition of expand_fast's dependent chain (VERDICT r02 "decompose the ~11 us
small-level floor"), from the diagnostic build (scripts/build_timeline.sh, SR_TIMELINE=1).

    python scripts/timeline.py [--model 2pc --n 9] [--checks 3]

Lane 0 of wave 0 of every workgroup stamps s_memrealtime (100 MHz, shared by every CU) after
draining its memory counters at each link (kernels.hpp SR_TL): 0 entry, 1 frontier size known
(the previous level's claims, one agent-scope load), 2 first parents loaded and their enabled
masks computed, 3 first successor map in LDS, 4 first probes returned, 5 first claims (CAS) done,
6 all chunks done, 7 stage span reserved (one device atomic), 8 stage written + properties,
9 exit. Per launch: its span (first entry .. last exit over all workgroups), the gap from the
previous launch's last exit, and the median workgroup's time per link.
"""
import argparse
import ctypes
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["SR_LIB_PATH"] = os.path.join(ROOT, "stateright_amd", "libstateright_gpu_timeline.so")
sys.path.insert(0, ROOT)

from stateright_amd import IncrementLock, Paxos, TwoPhaseSys  # noqa: E402
from stateright_amd import _native as N  # noqa: E402

TL_STAMPS, TL_BLOCKS, TL_LAUNCHES = 16, 2048, 64
TICK_US = 0.01  # s_memrealtime: 100 MHz
LINKS = ["size", "parents", "map", "probe", "claim", "chunks", "reserve", "write", "exit"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="2pc", choices=["2pc", "paxos", "increment_lock"])
    ap.add_argument("--n", type=int, default=9)
    ap.add_argument("--checks", type=int, default=3, help="warmup checks before the traced one")
    args = ap.parse_args()
    lib = N.load()
    lib.sr_timeline_reset.restype = ctypes.c_int64
    lib.sr_timeline_reset.argtypes = [ctypes.c_int32]
    lib.sr_timeline_fetch.restype = ctypes.c_int64
    lib.sr_timeline_fetch.argtypes = [ctypes.c_int32, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int64]
    make = {"2pc": lambda: TwoPhaseSys(args.n), "paxos": lambda: Paxos(args.n),
            "increment_lock": lambda: IncrementLock(args.n)}[args.model]
    hint = {"2pc": 6 ** args.n + 4 ** args.n + 2 ** args.n}.get(args.model, 0)

    def check():
        b = make().checker().order("fast")
        if hint:
            b = b.capacity_hint(hint)
        return b.spawn_bfs().join()

    for _ in range(args.checks):
        check()
    words = lib.sr_timeline_reset(0)
    assert words > 0, N.last_error()
    c = check()
    buf = (ctypes.c_uint64 * words)()
    assert lib.sr_timeline_fetch(0, buf, words) == words
    print(f"# {args.model} {args.n}: unique {c.unique_state_count()}, levels {c.stats()['levels']}")

    launches = []
    for L in range(TL_LAUNCHES):
        base = L * TL_BLOCKS * TL_STAMPS
        blocks = []
        for b in range(TL_BLOCKS):
            t = buf[base + b * TL_STAMPS: base + (b + 1) * TL_STAMPS]
            if t[0]:
                blocks.append(list(t))
        if blocks:
            launches.append(blocks)
    launches.sort(key=lambda bl: min(t[0] for t in bl))
    print("level  frontier  grid  span_us  gap_us  entry_skew  exit_skew | median link us: " + " ".join(f"{x:>7}" for x in LINKS))
    prev_end = None
    total = 0.0
    tails = []
    for i, bl in enumerate(launches):
        start = min(t[0] for t in bl)
        end = max(t[9] for t in bl)
        work = [t for t in bl if t[1]]  # expanding workgroups (the service workgroup stops at entry)
        meta = bl[0][TL_STAMPS - 1]
        grid, fr = meta >> 32, meta & 0xFFFFFFFF
        span = (end - start) * TICK_US
        total += span
        gap = (start - prev_end) * TICK_US if prev_end else 0.0
        prev_end = end
        med = []
        for k in range(1, 10):
            d = [(t[k] - t[k - 1]) * TICK_US for t in work if t[k] and t[k - 1]]
            med.append(statistics.median(d) if d else float("nan"))
        # inside "map": 2 -> 10 self-loops + parent stage, 10 -> 11 wave scan, 11 -> 12 map loop, 12 -> 3 LDS sync
        sub = []
        for a, b in ((2, 10), (10, 11), (11, 12), (12, 3)):
            d = [(t[b] - t[a]) * TICK_US for t in work if t[a] and t[b]]
            sub.append(statistics.median(d) if d else float("nan"))
        entry_skew = (statistics.median([t[0] for t in bl]) - start) * TICK_US
        exit_skew = (end - statistics.median([t[9] for t in bl if t[9]])) * TICK_US
        # the reservation link (one device atomic on the level's single claims line) across workgroups:
        # p90 and max, and when the chunks of the workgroups ended (p10 / p90 after the launch start)
        res = sorted((t[7] - t[6]) * TICK_US for t in work if t[7] and t[6])
        ends = sorted((t[6] - start) * TICK_US for t in work if t[6])
        q = lambda v, f: v[min(len(v) - 1, int(f * len(v)))] if v else float("nan")
        tails.append(f"{i:5d} reserve p90 {q(res, 0.9):6.2f} max {q(res, 1.0):6.2f} | chunks end p10 {q(ends, 0.1):6.1f} "
                     f"p50 {q(ends, 0.5):6.1f} p90 {q(ends, 0.9):6.1f} max {q(ends, 1.0):6.1f} us")
        # by workgroup index (the array index is blockIdx.x): quarters of the grid, entry and chunk end
        nb = len(bl)
        for qi in range(4):
            part = [t for b, t in enumerate(bl) if t[1] and qi * nb // 4 <= b < (qi + 1) * nb // 4]
            if not part:
                continue
            st = sorted((t[0] - start) * TICK_US for t in part)
            en = sorted((t[6] - start) * TICK_US for t in part if t[6])
            ch = sorted((t[6] - t[5]) * TICK_US for t in part if t[6] and t[5])
            tails.append(f"        q{qi}: entry p50 {q(st, 0.5):6.1f} max {q(st, 1.0):6.1f} | chunk end p50 {q(en, 0.5):6.1f} "
                         f"max {q(en, 1.0):6.1f} | chunks link p50 {q(ch, 0.5):6.1f} p90 {q(ch, 0.9):6.1f}")
        print(f"{i:5d} {fr:9d} {grid:5d} {span:8.1f} {gap:7.1f} {entry_skew:11.1f} {exit_skew:10.1f} | " +
              "                 " + " ".join(f"{x:7.2f}" for x in med) + "  | map: " + " ".join(f"{x:5.2f}" for x in sub))
    print(f"# sum of spans {total:.1f} us over {len(launches)} launches")
    print("\n".join(tails))


if __name__ == "__main__":
    main()
