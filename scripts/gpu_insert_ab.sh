#!/bin/bash
# Partitioned insert A/B: the in-tree engine (probe-batched insert) against build_ab/lib_head.so,
# x SR_INSERT_GRID; summed kernel time per check of 2pc N=11 / N=9 over T virtual partitions.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/insert_ab
mkdir -p "$O"
timeout -k 10 400 python -u -m pytest tests/test_gpu_partitioned.py tests/test_gpu_dist_ranks.py -x -q --timeout 300 --timeout-method thread > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
tail -1 "$O/tests.log"
for N in 9 11; do for T in 2 4; do for v in head new; do for g in 4096; do
  lib=stateright_amd/libstateright_gpu.so; [ $v = head ] && lib=build_ab/lib_head.so
  sc=4; [ $v = nosent ] && sc=0
  d=$O/${v}_g${g}_t${T}_n$N
  SR_SEND_CACHE=$sc SR_LIB_PATH=$lib SR_INSERT_GRID=$g timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o t -- python3 scripts/prof_partitioned.py virtual $T $N 2 > $d.log 2>&1 || { echo "fail $d"; tail -5 $d.log; exit 1; }
  python3 - "$d/t_kernel_stats.csv" "$v g$g T$T N$N" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = {}
for r in rows:
    k = r["Name"].split("<")[0].split("(")[0].replace("void ", "").replace("sr::", "")
    tot[k] = tot.get(k, 0) + float(r["TotalDurationNs"]) / 3e6  # 3 checks -> ms per check
print(sys.argv[2], open(sys.argv[1].rsplit("/", 1)[0] + ".log").read().strip().splitlines()[-1].split("records_routed")[-1].strip(), "ms/check:", {k: round(v, 2) for k, v in sorted(tot.items(), key=lambda x: -x[1])[:4]}, "sum", round(sum(tot.values()), 2))
PY
done; done; done; done
