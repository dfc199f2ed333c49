"""Every dispatch of the last check in a rocprofv3 kernel-trace CSV: short name, duration, gap."""
import csv
import re
import sys

for path in sys.argv[1:]:
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    roots = [i for i, r in enumerate(rows) if "insert_roots" in r["Kernel_Name"]]
    tail = rows[roots[-1]:]
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in tail) / 1e3
    span = (int(tail[-1]["End_Timestamp"]) - int(tail[0]["Start_Timestamp"])) / 1e3
    print(f"{path}: kernels={len(tail)} busy={busy:.0f}us span={span:.0f}us")
    out, prev = [], None
    for r in tail:
        name = re.sub(r"^(void )?sr::", "", r["Kernel_Name"]).split("<")[0].split("(")[0]
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        g = (int(r["Start_Timestamp"]) - prev) / 1e3 if prev else 0
        prev = int(r["End_Timestamp"])
        out.append(f"{name[:14]}:{d:.0f}(+{g:.0f})")
    print("  " + " ".join(out))
