"""Summary of scripts/pmc_inflight.sh: for expand_fast dispatches of >= 100 us (the big levels),
resident waves per CU, outstanding VMEM instructions per wave and per CU, the mean L1->L2 read
latency, and the memory-side read request rate; Little's law then says how many requests the
chip keeps in flight against how many the measured request ceiling needs."""
import collections
import csv
import glob
import sys

O = sys.argv[1]
CUS, CLK = 256, 2.4e9
EA_READ_CEIL = 60.5e9  # profiles/pmc_ceiling.json: memory-side read requests/s (random 8-B loads)
for n in (9, 11):
    files = glob.glob(f"{O}/n{n}/*counter_collection.csv")
    if not files:
        continue
    per = collections.defaultdict(dict)
    dur = {}
    for r in csv.DictReader(open(files[0])):
        if "expand_fast" not in r["Kernel_Name"] or "true>" in r["Kernel_Name"]:
            continue
        per[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
        dur[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    big = [d for d in per if dur[d] >= 100_000]
    tot = collections.defaultdict(float)
    for d in big:
        for k, v in per[d].items():
            tot[k] += v
    ns = sum(dur[d] for d in big)
    cyc = ns * 1e-9 * CLK
    waves_cu = tot["SQ_WAVE_CYCLES"] / max(1.0, cyc) / CUS
    vmem_cu = tot["SQ_INST_LEVEL_VMEM"] / max(1.0, cyc) / CUS
    lat = tot["TCP_TCC_READ_REQ_LATENCY_sum"] / max(1.0, tot["TCP_TCC_READ_REQ_sum"])
    ea_rate = tot["TCC_EA0_RDREQ_sum"] / (ns * 1e-9)
    l2_rate = tot["TCP_TCC_READ_REQ_sum"] / (ns * 1e-9)
    print(f"2pc N={n}: {len(big)} big dispatches, {ns / 1e6:.2f} ms")
    print(f"  resident waves per CU {waves_cu:.1f} (SQ_WAVE_CYCLES / cycles / CUs; raw counter units); "
          f"VMEM instructions outstanding per CU {vmem_cu:.1f}, per wave {vmem_cu / max(waves_cu, 1e-9):.2f}")
    print(f"  L1->L2 reads {l2_rate / 1e9:.1f} G/s at {lat:.0f} cycles mean latency -> {l2_rate * lat / CLK:.0f} in flight (Little)")
    print(f"  memory-side reads {ea_rate / 1e9:.1f} G/s = {ea_rate / EA_READ_CEIL:.2f} of the {EA_READ_CEIL / 1e9:.1f} G/s ceiling; "
          f"at that latency the ceiling needs {EA_READ_CEIL * lat / CLK:.0f} in flight")
