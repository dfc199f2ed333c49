"""Summary of scripts/pmc_inflight.sh over expand_fast dispatches of >= 100 us (the big levels):
resident waves per CU, vector-memory instructions outstanding, memory-side read requests in
flight (their per-cycle level) and the latency Little's law gives them, beside how many the
measured request ceiling would need at that latency; and the L1 address-translation miss rate."""
import collections
import csv
import glob
import sys
import os
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from kname import is_timed_expand  # noqa: E402

O = sys.argv[1]
CUS = 256
EA_READ_CEIL = 60.5e9  # profiles/pmc_ceiling.json: memory-side read requests/s (random 8-B loads)


def load(n, p):
    files = glob.glob(f"{O}/n{n}_{p}/*counter_collection.csv")
    per = collections.defaultdict(dict)
    dur = {}
    if not files:
        return per, dur
    for r in csv.DictReader(open(files[0])):
        if not is_timed_expand(r["Kernel_Name"]):
            continue
        per[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
        dur[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return per, dur


def big_sums(n, p):
    per, dur = load(n, p)
    big = [d for d in per if dur[d] >= 100_000]
    tot = collections.defaultdict(float)
    for d in big:
        for k, v in per[d].items():
            tot[k] += v
    return tot, sum(dur[d] for d in big), len(big)


for n in (9, 11):
    a, ns_a, k = big_sums(n, "A")
    b, ns_b, _ = big_sums(n, "B")
    c, ns_c, _ = big_sums(n, "C")
    if not k:
        continue
    # GRBM_GUI_ACTIVE is summed over the 8 XCDs: one XCD's cycles are 1/8 of it
    xcd = max(1, round(b["GRBM_GUI_ACTIVE"] / (ns_b * 1e-9) / 2.4e9)) if b["GRBM_GUI_ACTIVE"] else 8
    cyc_a = (a["GRBM_GUI_ACTIVE"] or ns_a * 2.4 * xcd) / xcd
    cyc_b = (b["GRBM_GUI_ACTIVE"] or ns_b * 2.4 * xcd) / xcd
    clk = cyc_b / (ns_b * 1e-9)  # one XCD's cycles per second
    print(f"2pc N={n}: {k} big dispatches, {ns_a / 1e6:.2f} ms (pass A), clock {clk / 1e9:.2f} GHz, {xcd} XCDs")
    # SQ_WAVE_CYCLES counts in quad-cycles (x4): resident waves per CU
    print(f"  resident waves per CU {4 * a['SQ_WAVE_CYCLES'] / cyc_a / CUS:.1f} (SQ_WAVE_CYCLES x 4 / cycles / CUs), "
          f"waves launched {a['SQ_WAVES']:.3g}; VMEM instructions {a['SQ_INSTS_VMEM']:.3g}")
    inflight = b["TCC_EA0_RDREQ_LEVEL_sum"] / cyc_b
    rate = b["TCC_EA0_RDREQ_sum"] / (ns_b * 1e-9)
    lat = inflight / rate * 1e9 if rate else 0.0
    print(f"  memory-side reads: {rate / 1e9:.1f} G/s = {rate / EA_READ_CEIL:.2f} of the {EA_READ_CEIL / 1e9:.1f} G/s ceiling; "
          f"{inflight:.0f} in flight -> {lat:.0f} ns each (Little); the ceiling at that latency needs "
          f"{EA_READ_CEIL * lat * 1e-9:.0f} in flight")
    req = c["TCP_UTCL1_TRANSLATION_MISS_sum"] + c["TCP_UTCL1_TRANSLATION_HIT_sum"]
    if req:
        print(f"  UTCL1 translations: {req:.3g}, miss rate {c['TCP_UTCL1_TRANSLATION_MISS_sum'] / req:.3f}; "
              f"stall cycles: in-flight max {c['TCP_UTCL1_STALL_INFLIGHT_MAX_sum']:.3g}, multi-miss "
              f"{c['TCP_UTCL1_STALL_MULTI_MISS_sum']:.3g}")
