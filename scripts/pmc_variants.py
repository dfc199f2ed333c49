"""Summary of scripts/pmc_variants.sh: per engine setting, expand_fast's big launches (>= 100 us):
time, wave-instructions (VALU / SALU / LDS / VMEM), the fraction of wave-cycles waiting, resident
waves per CU, and the memory-side read requests (rate, in flight, Little's-law latency)."""
import collections
import csv
import glob
import sys
import os
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from kname import is_timed_expand  # noqa: E402

O, ENVS = sys.argv[1], sys.argv[2:]
CUS = 256


def big(i, p):
    files = glob.glob(f"{O}/v{i}_{p}/*counter_collection.csv")
    per, dur = collections.defaultdict(dict), {}
    for f in files:
        for r in csv.DictReader(open(f)):
            if not is_timed_expand(r["Kernel_Name"]):
                continue
            per[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
            dur[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    ids = [d for d in per if dur[d] >= 100_000]
    tot = collections.defaultdict(float)
    for d in ids:
        for k, v in per[d].items():
            tot[k] += v
    return tot, sum(dur[d] for d in ids), len(ids)


for i, env in enumerate(ENVS):
    a, ns_a, k = big(i, "A")
    b, ns_b, _ = big(i, "B")
    if not k:
        print(f"[{env}] no big launches")
        continue
    xcd = 8
    cyc_a = (a["GRBM_GUI_ACTIVE"] or ns_a * 2.4 * xcd) / xcd
    cyc_b = (b["GRBM_GUI_ACTIVE"] or ns_b * 2.4 * xcd) / xcd
    waves = 4 * a["SQ_WAVE_CYCLES"] / cyc_a / CUS
    rate = b["TCC_EA0_RDREQ_sum"] / (ns_b * 1e-9)
    inflight = b["TCC_EA0_RDREQ_LEVEL_sum"] / cyc_b
    lat = inflight / rate * 1e9 if rate else 0.0
    print(f"[{env or 'default'}] {k} big launches {ns_a / 1e6:.3f} ms (pass A) {ns_b / 1e6:.3f} ms (pass B); "
          f"VALU {a['SQ_INSTS_VALU']:.3g} SALU {a['SQ_INSTS_SALU']:.3g} LDS {a['SQ_INSTS_LDS']:.3g} "
          f"VMEM {a['SQ_INSTS_VMEM']:.3g}; wait {a['SQ_WAIT_ANY'] / max(1, a['SQ_WAVE_CYCLES']):.2f} of wave-cycles; "
          f"resident waves/CU {waves:.1f}; EA reads {rate / 1e9:.1f} G/s, {inflight:.0f} in flight, {lat:.0f} ns; "
          f"EA writes {b['TCC_EA0_WRREQ_sum'] / (ns_b * 1e-9) / 1e9:.1f} G/s, atomics {b['TCC_EA0_ATOMIC_sum'] / (ns_b * 1e-9) / 1e9:.1f} G/s")
