"""Kernel time vs span of the last full check in a rocprofv3 kernel trace (gaps = host/launch idle)."""
import csv
import sys

for path in sys.argv[1:]:
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    roots = [i for i, r in enumerate(rows) if "insert_roots" in r["Kernel_Name"]]
    tail = rows[roots[-1]:]
    ex = [r for r in tail if "expand" in r["Kernel_Name"]]
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in tail) / 1e3
    span = (int(tail[-1]["End_Timestamp"]) - int(tail[0]["Start_Timestamp"])) / 1e3
    gaps = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 for a, b in zip(ex, ex[1:])]
    print(f"{path}: kernels={len(tail)} expand={len(ex)} busy={busy:.0f}us span={span:.0f}us "
          f"expand-gaps sum={sum(gaps):.0f}us max={max(gaps):.0f}us")
    print("  durations:", " ".join(f"{(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3:.0f}" for r in ex))
    print("  gaps:     ", " ".join(f"{g:.0f}" for g in gaps))
