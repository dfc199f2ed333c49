"""Prints the last step's expand dispatches (duration, grid) from a rocprofv3 kernel-trace CSV."""
import csv
import sys

for path in sys.argv[1:]:
    rows = list(csv.DictReader(open(path)))
    ex = [r for r in rows if "expand" in r["Kernel_Name"] or "scatter" in r["Kernel_Name"]]
    # the last step = dispatches after the last insert_roots
    roots = [i for i, r in enumerate(rows) if "insert_roots" in r["Kernel_Name"]]
    tail = [r for r in rows[roots[-1]:] if r in ex] if roots else ex
    tot = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in tail) / 1e3
    print(path, f"launches={len(tail)} total={tot:.1f}us")
    print("  " + " ".join(f'{(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3:.0f}/{int(r["Grid_Size_X"]) // 64}w'
                          for r in tail))
