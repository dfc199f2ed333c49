"""Median per-dispatch duration and preceding idle gap over the timed (non-counting) checks of a
rocprofv3 kernel trace of bench.py (scripts/ktrace.sh): per dispatch index "dur/gap" in us.
    python3 scripts/ktrace_median.py <trace_kernel_trace.csv>"""
import csv
import statistics as st
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "roots" in r["Kernel_Name"]] + [len(rows)]
G, D, spans = {}, {}, []
for c in range(len(starts) - 1):
    chk = rows[starts[c]:starts[c + 1]]
    if any("true, " in r["Kernel_Name"] for r in chk):  # the counting pass (STATS instantiation)
        continue
    prev = None
    for i, r in enumerate(chk):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if prev is not None:
            G.setdefault(i, []).append((s - prev) / 1e3)
        D.setdefault(i, []).append((e - s) / 1e3)
        prev = e
    spans.append((int(chk[-1]["Start_Timestamp"]) - int(chk[0]["Start_Timestamp"])) / 1e3)
print(f"{len(spans)} checks; median span (first start .. last start) {st.median(spans):.1f} us")
print(" ".join(f"{i}:{st.median(D[i]):.1f}/{st.median(G.get(i, [0])):.1f}" for i in sorted(D)))
print(f"sum of median gaps {sum(st.median(v) for v in G.values()):.1f} us, of median durations {sum(st.median(v) for v in D.values()):.1f} us")
