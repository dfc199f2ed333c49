#!/bin/bash
# Round 6: where config 4's route kernel spends its time against expand_fast on the same state space
# (2pc N=11): instruction mix, occupancy, waits and memory-side requests, per kernel family summed
# over its dispatches (two PMC passes per run, counters with --kernel-trace only).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06pmc_c4
mkdir -p $O
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
B="TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_ATOMIC_sum GRBM_GUI_ACTIVE"
for p in A B; do
  timeout -s KILL 240 rocprofv3 --pmc ${!p} --kernel-trace --output-format csv -d $O/part_$p -o p -- python3 scripts/prof_partitioned.py virtual 8 11 1 > $O/part_$p.log 2>&1 || { echo "part $p failed"; tail -3 $O/part_$p.log; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc ${!p} --kernel-trace --output-format csv -d $O/one_$p -o p -- python3 bench.py --rm-count 11 --steps 1 --warmup 1 --cpu-baseline 0 --config4-steps 0 --no-hint-steps 0 > $O/one_$p.log 2>&1 || { echo "one $p failed"; tail -3 $O/one_$p.log; exit 1; }
done
python3 - $O <<'PY'
import csv, glob, sys, collections
O = sys.argv[1]
def fam(k):
    for f in ("expand_route", "insert_recv", "expand_fast"):
        if f in k: return f
    return None
res = collections.defaultdict(lambda: collections.defaultdict(float))
dur = collections.defaultdict(float)
for run in ("part", "one"):
    for p in ("A", "B"):
        fs = glob.glob(f"{O}/{run}_{p}/*counter_collection.csv")
        seen = set()
        for r in csv.DictReader(open(fs[0])):
            f = fam(r["Kernel_Name"])
            if not f: continue
            key = (run, f)
            res[key][r["Counter_Name"]] += float(r["Counter_Value"])
            if p == "A" and (r["Dispatch_Id"]) not in seen:
                seen.add(r["Dispatch_Id"])
                dur[key] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
for key, c in sorted(res.items()):
    ns = dur[key]
    cyc = c["GRBM_GUI_ACTIVE"] / 8 if c["GRBM_GUI_ACTIVE"] else ns * 2.4
    print(f"{key[0]:4s} {key[1]:12s} {ns/1e6:8.2f} ms  VALU {c['SQ_INSTS_VALU']:.3g} SALU {c['SQ_INSTS_SALU']:.3g} LDS {c['SQ_INSTS_LDS']:.3g} "
          f"VMEM {c['SQ_INSTS_VMEM']:.3g} wait {c['SQ_WAIT_ANY']/max(1,c['SQ_WAVE_CYCLES']):.2f} busy-waves/CU {4*c['SQ_WAVE_CYCLES']/max(1,cyc)/256:.1f} "
          f"EA rd {c['TCC_EA0_RDREQ_sum']:.3g} wr {c['TCC_EA0_WRREQ_sum']:.3g} at {c['TCC_EA0_ATOMIC_sum']:.3g}")
PY
