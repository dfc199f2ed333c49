#!/bin/bash
# Instruction mix of expand_fast on paxos (the round-3 verdict's "VALU per successor"): one PMC
# pass (SQ_ counters only, --kernel-trace) over bench.py, the non-counting dispatches summed and
# divided by the checks they cover and the check's successors.
#   scripts/pmc_valu_paxos.sh [clients launches_per_check successors_per_check]   (default 3 29 2420477)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
C=${1:-3}; LPC=${2:-29}; SPC=${3:-2420477}
O=gpurun_out/pmc_valu_paxos_c$C
mkdir -p $O
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM --kernel-trace --output-format csv -d $O/p3 -o p -- python3 bench.py --model paxos --clients $C --steps 3 --warmup 1 --cpu-baseline 0 --config4-steps 0 --no-hint-steps 0 > $O/p3.log 2>&1 || { echo "pmc failed"; tail -3 $O/p3.log; exit 1; }
python3 - $O $C $LPC $SPC <<'PY'
import csv, glob, sys, collections
sys.path.insert(0, 'scripts')
from kname import is_timed_expand
O, C, LPC, SPC = sys.argv[1], int(sys.argv[2]), float(sys.argv[3]), float(sys.argv[4])
(f,) = glob.glob(f"{O}/p3/*counter_collection.csv")
per = collections.defaultdict(dict)
dur = {}
for r in csv.DictReader(open(f)):
    if not is_timed_expand(r["Kernel_Name"]):
        continue
    per[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
    dur[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
tot = collections.defaultdict(float)
for d in per.values():
    for k, v in d.items():
        tot[k] += v
checks = len(per) / LPC
succ = checks * SPC
print(f"paxos C={C}: {len(per)} dispatches (~{checks:.1f} checks), {sum(dur.values())/1e6:.3f} ms under PMC")
for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM"):
    print(f"  {k}: {tot[k]:.4g} wave-instructions, {tot[k]/succ:.2f} per successor")
print(f"  waits: SQ_WAIT_ANY / SQ_WAVE_CYCLES = {tot['SQ_WAIT_ANY']/max(tot['SQ_WAVE_CYCLES'],1):.2f}; active issue / wave-cycles = {tot['SQ_ACTIVE_INST_ANY']/max(tot['SQ_WAVE_CYCLES'],1):.2f}")
PY
