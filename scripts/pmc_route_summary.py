"""Per-successor counters of expand_route (2 virtual partitions) vs expand_fast (one partition) from
scripts/gpu_pmc_route.sh: counter totals per kernel, divided by the checks profiled."""
import collections
import csv
import glob
import os
import sys

base = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmcr"
checks = 3  # warmup + 2
for cfg in ("virtual1", "virtual2"):
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    for path in glob.glob(os.path.join(base, cfg + "_p*", "*counter_collection.csv")):
        for r in csv.DictReader(open(path)):
            k = r["Kernel_Name"]
            k = "expand_route" if "expand_route" in k else "expand_fast" if "expand_fast" in k else \
                "insert_recv" if "insert_recv" in k else None
            if k:
                tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, c in sorted(tot.items()):
        print(f"== {cfg} {k}")
        for name, v in sorted(c.items()):
            print(f"   {name:28s} {v / checks:16.4g} per check")
