#!/bin/bash
# Atomic / read-request counts of the expand kernel per probe-load policy.
set -e
export TMPDIR=/tmp
for pol in 0 1 2 3; do
  SR_PROBE_LOAD=$pol REPS=2 timeout -k 10 120 rocprofv3 --pmc TCC_EA0_ATOMIC_sum TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d gpurun_out/pol$pol -o pol -- python3 scripts/prof_driver.py > gpurun_out/pol$pol.log 2>&1
  python3 - $pol <<'PY'
import csv,sys,collections
pol=sys.argv[1]
rows=list(csv.DictReader(open(f'gpurun_out/pol{pol}/pol_counter_collection.csv')))
ex=[r for r in rows if 'expand_fast' in r['Kernel_Name']]
d=sorted(set(int(r['Dispatch_Id']) for r in ex)); last=set(d[len(d)//2:])
t=collections.defaultdict(float)
for r in ex:
    if int(r['Dispatch_Id']) in last: t[r['Counter_Name']]+=float(r['Counter_Value'])
print("pol",pol,{k:f"{v:.4g}" for k,v in t.items()})
PY
done
