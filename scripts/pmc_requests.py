#!/usr/bin/env python3
"""Summarises scripts/gpu_roofline.sh's PMC passes into profiles/pmc_ceiling.json and
profiles/pmc_traffic.json (both stamped with the engine's source digest)."""
import collections
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from stateright_amd.build import source_digest  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from kname import is_timed_expand  # noqa: E402

LABELS = {"2pc9": "2pc N=9", "2pc10": "2pc N=10", "2pc11": "2pc N=11", "inclock10": "increment_lock N=10",
          "inclock11": "increment_lock N=11", "paxos3": "paxos C=3"}


def dispatches(d, want=None):
    """{dispatch id: (kernel name, ns, {counter: value})} of the counter CSV under directory d."""
    (path,) = glob.glob(os.path.join(d, "*counter_collection.csv"))
    out = {}
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if want and not want(name):
            continue
        k = out.setdefault(r["Dispatch_Id"], [name, int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), {}])
        k[2][r["Counter_Name"]] = float(r["Counter_Value"])
    return out


def expand(name):  # the timed expand kernel (not the counting instantiation, STATS = true)
    return is_timed_expand(name)


def main(o):
    stamp = {"source_digest": source_digest()}
    try:
        stamp["commit"] = subprocess.run(["git", "rev-parse", "--short=12", "HEAD"], cwd=ROOT, capture_output=True,
                                         text=True).stdout.strip() or None
    except OSError:
        stamp["commit"] = None
    ceil = collections.defaultdict(float)
    rows = []
    for _, (name, ns, c) in dispatches(os.path.join(o, "ceiling")).items():
        if ns < 20000 or not any(k in name for k in ("rand_", "mix")):
            continue
        rates = {k: c.get(k, 0.0) / ns * 1e9 for k in ("TCC_EA0_RDREQ_sum", "TCC_EA0_WRREQ_sum", "TCC_EA0_ATOMIC_sum")}
        rows.append({"kernel": name.split("(")[0], "us": ns / 1e3, **{k + "_per_s": v for k, v in rates.items()}})
        for k, v in rates.items():
            ceil[k] = max(ceil[k], v)
    ceiling = {**stamp, "source": "scripts/microbench_random.hip under rocprofv3 --pmc " +
               "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_ATOMIC_sum (scripts/gpu_roofline.sh)",
               "ea_read_req_per_s": ceil["TCC_EA0_RDREQ_sum"], "ea_write_req_per_s": ceil["TCC_EA0_WRREQ_sum"],
               "ea_atomic_req_per_s": ceil["TCC_EA0_ATOMIC_sum"], "dispatches": rows}
    configs = {}
    for tag, label in LABELS.items():
        if not os.path.isdir(os.path.join(o, tag)):
            continue
        req = dispatches(os.path.join(o, tag, "req"), expand)
        rd = dispatches(os.path.join(o, tag, "rd"), expand)
        wr = dispatches(os.path.join(o, tag, "wr"), expand)
        n = len(req)
        s = lambda D, k: sum(v[2].get(k, 0.0) for v in D.values())  # noqa: E731
        ns = sum(v[1] for v in req.values())
        read_bytes = (s(rd, "TCC_EA0_RDREQ_128B_sum") * 128 + s(rd, "TCC_EA0_RDREQ_64B_sum") * 64 +
                      s(rd, "TCC_EA0_RDREQ_32B_sum") * 32) / max(1, len(rd))
        write_bytes = s(wr, "WRITE_SIZE") * 1024 / max(1, len(wr))
        configs[label] = {
            "launches": n, "kernel": next(iter(req.values()))[0].split("(")[0] if req else None,
            "ea_read_req_per_launch": s(req, "TCC_EA0_RDREQ_sum") / n,
            "ea_write_req_per_launch": s(req, "TCC_EA0_WRREQ_sum") / n,
            "ea_atomic_req_per_launch": s(req, "TCC_EA0_ATOMIC_sum") / n,
            "read_bytes_per_launch": read_bytes, "write_bytes_per_launch": write_bytes,
            "bytes_per_launch": read_bytes + write_bytes,
            "avg_launch_us_under_pmc": ns / n / 1e3,
        }
    traffic = {**stamp, "note": "beyond-L2 (Infinity Cache + HBM) requests and bytes per expand_fast launch, averaged "
               "over every non-counting expand_fast dispatch of `bench.py --steps 1 --warmup 1` (scripts/gpu_roofline.sh); "
               "read bytes from TCC_EA0_RDREQ_{128B,64B,32B} (FETCH_SIZE tallies 128-B requests at 64 B on gfx950), "
               "write bytes from WRITE_SIZE", "configs": configs}
    for name, obj in (("pmc_ceiling.json", ceiling), ("pmc_traffic.json", traffic)):
        for d in (os.path.join(ROOT, "profiles"), o):
            with open(os.path.join(d, name), "w") as f:
                json.dump(obj, f, indent=1)
    print(json.dumps({k: v for k, v in ceiling.items() if k != "dispatches"}))
    for label, c in configs.items():
        print(label, json.dumps(c))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "roofline"))
