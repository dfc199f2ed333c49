#!/bin/bash
# Where expand_route's time goes at T = 8 (2pc N=11, virtual partitions): SQ counters per dispatch,
# in passes of their own (counters only with --kernel-trace).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/pmc_route
mkdir -p $O
timeout -k 10 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $line --kernel-trace --output-format csv -d $O/p$i -o p -- python3 scripts/prof_partitioned.py virtual 8 11 1 > $O/p$i.log 2>&1 || { echo "pass $i failed: $line"; tail -3 $O/p$i.log; continue; }
  echo "pass $i ok: $line"
done <<'PASSES'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS
SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_INST_LEVEL_LDS SQ_INST_LEVEL_VMEM
PASSES
python3 - $O <<'PY'
import csv, glob, sys, collections
O = sys.argv[1]
for d in sorted(glob.glob(O + "/p*/")):
    fs = glob.glob(d + "*counter_collection.csv")
    if not fs:
        continue
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(fs[0])):
        k = r["Kernel_Name"].split("(")[0].replace("void sr::", "")[:34]
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, c in tot.items():
        if "expand_route" in k or "insert_recv_lag<sr::TwoPhase, 4>" in k:
            print(d.split("/")[-2], k, {n: f"{v:.4g}" for n, v in c.items()})
PY
