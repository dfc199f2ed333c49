#!/bin/bash
# Memory type / load policy of random probes: timings, then the L2's memory-side request sizes per
# dispatch (one PMC pass; counters only with --kernel-trace).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/mtype
mkdir -p $O
timeout -k 10 120 ./scripts/microbench_mtype | tee $O/times.txt || exit 1
timeout -k 10 120 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum --kernel-trace --output-format csv -d $O/pmc -o p -- ./scripts/microbench_mtype > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
python3 - $O/pmc <<'PY'
import csv, glob, sys, collections
(path,) = glob.glob(sys.argv[1] + "/*counter_collection.csv")
d = collections.OrderedDict()
for r in csv.DictReader(open(path)):
    k = (r["Dispatch_Id"], r["Kernel_Name"].split("(")[0])
    d.setdefault(k, {})[r["Counter_Name"]] = float(r["Counter_Value"])
for (i, name), c in d.items():
    tot = c.get("TCC_EA0_RDREQ_sum", 0)
    print(f"{i:>4} {name:40s} rdreq {tot:12.4g}  32B {c.get('TCC_EA0_RDREQ_32B_sum',0):10.4g}  64B {c.get('TCC_EA0_RDREQ_64B_sum',0):10.4g}  128B {c.get('TCC_EA0_RDREQ_128B_sum',0):10.4g}")
PY
