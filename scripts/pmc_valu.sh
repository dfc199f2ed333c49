#!/bin/bash
# Instruction mix of expand_fast (single GPU, 2pc N=9 and N=11): VALU / SALU / LDS / VMEM wave-
# instructions and wave-cycles per dispatch, one PMC pass per configuration.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/pmc_valu
mkdir -p $O
for n in 9 11; do
  timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM --kernel-trace --output-format csv -d $O/n$n -o p -- python3 bench.py --rm-count $n --steps 1 --warmup 1 --cpu-baseline 0 --config4-steps 0 > $O/n$n.log 2>&1 || { echo "n$n failed"; tail -3 $O/n$n.log; exit 1; }
done
python3 - $O <<'PY'
import csv, glob, sys, collections
sys.path.insert(0, 'scripts')
from kname import is_timed_expand
O = sys.argv[1]
for n in (9, 11):
    (f,) = glob.glob(f"{O}/n{n}/*counter_collection.csv")
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
    ns = sum(dur.values())
    cap = ns * 1e-9 * 256 * 4 * 2.4e9 / 4  # wave64 VALU instructions the chip can issue in that time
    print(f"2pc N={n}: {len(per)} dispatches, {ns/1e6:.2f} ms; VALU {tot['SQ_INSTS_VALU']:.3g} ({tot['SQ_INSTS_VALU']/cap:.2f} of issue capacity), "
          f"SALU {tot['SQ_INSTS_SALU']:.3g}, LDS {tot['SQ_INSTS_LDS']:.3g}, VMEM {tot['SQ_INSTS_VMEM']:.3g}, "
          f"wait {tot['SQ_WAIT_ANY']/tot['SQ_WAVE_CYCLES']:.2f} of wave-cycles, active {tot['SQ_ACTIVE_INST_ANY']/tot['SQ_WAVE_CYCLES']:.2f}")
PY
