"""Sums rocprofv3 counter-collection CSVs per kernel name (first 40 chars)."""
import collections
import csv
import glob
import sys

tot = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for path in glob.glob(sys.argv[1] + "/*/*counter_collection.csv"):
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"][:40]
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add((path, r["Dispatch_Id"]))
for k, d in tot.items():
    print(k, "dispatches", len(disp[k]))
    for c, v in sorted(d.items()):
        print(f"   {c:28s} {v:16.0f}")
