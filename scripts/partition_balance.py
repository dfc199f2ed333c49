"""Per-partition kernel time of a partitioned search traced with rocprofv3 --kernel-trace on one GPU
(virtual partitions: every level launches expand_route then insert_recv_lag once per partition, in
partition order). Prints the summed kernel time, the per-partition sums and the critical-path
estimate sum over levels of max over partitions (route + insert) that T GPUs would see.
    python scripts/partition_balance.py <kernel_trace.csv> <T> <checks>"""
import csv
import sys

path, T, checks = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
route = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows if "expand_route" in r["Kernel_Name"]]
insert = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows if "insert_recv" in r["Kernel_Name"]]
other = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows
            if "expand_route" not in r["Kernel_Name"] and "insert_recv" not in r["Kernel_Name"])
assert len(route) % T == 0 and len(insert) % T == 0, (len(route), len(insert))
L = len(route) // T
per_part = [0.0] * T
crit = 0.0
for lv in range(L):
    w = [route[lv * T + p] + (insert[lv * T + p] if lv * T + p < len(insert) else 0) for p in range(T)]
    for p in range(T):
        per_part[p] += w[p]
    crit += max(w)
tot = sum(route) + sum(insert)
ms = lambda ns: ns / 1e6 / checks  # noqa: E731
print(f"T={T} per check: route {ms(sum(route)):.2f} ms, insert {ms(sum(insert)):.2f} ms, other {ms(other):.2f} ms; "
      f"route+insert per partition mean {ms(tot / T):.2f} max {ms(max(per_part)):.2f} ms; "
      f"critical path (sum of per-level max) {ms(crit):.2f} ms")
