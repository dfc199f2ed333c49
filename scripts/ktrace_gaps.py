"""Per-level kernel durations and the idle gap before each launch, from a rocprofv3 kernel trace of
bench.py (scripts/ktrace.sh): the last complete check (dispatches after the last roots launch).
    python3 scripts/ktrace_gaps.py gpurun_out/<dir>/.../trace_kernel_trace.csv [check index, -1 = last]
(bench.py's last check is its counting pass, SR stats on: -2 is the last timed one.)
"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "roots" in r["Kernel_Name"]] + [len(rows)]
k = int(sys.argv[2]) if len(sys.argv) > 2 else -1
chk = rows[starts[k - 1]:starts[k]]
prev_end = None
tot_k = tot_g = 0.0
print(" idx  dur_us  gap_us  grid  kernel")
for i, r in enumerate(chk):
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    g = (s - prev_end) / 1e3 if prev_end is not None else 0.0
    d = (e - s) / 1e3
    tot_k += d
    tot_g += max(g, 0.0)
    prev_end = e
    name = r["Kernel_Name"].split("(")[0][:60]
    print(f"{i:4d} {d:7.1f} {g:7.1f} {int(r['Grid_Size_X']) // 256:5d}  {name}")
print(f"check span {(int(chk[-1]['End_Timestamp']) - int(chk[0]['Start_Timestamp'])) / 1e3:.1f} us: kernels {tot_k:.1f} us, gaps {tot_g:.1f} us over {len(chk)} dispatches")
