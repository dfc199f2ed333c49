#!/bin/bash
# Kernel traces of 2pc N: the single-GPU engine (expand_fast) and the partitioned engine on ONE
# partition (expand_route, no records), one warmup + one traced check each, per-level durations.
#   scripts/gpu_route_vs_fast.sh <N>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/rvf
N=$1
N=$N REPS=2 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/rvf/fast -o t -- python3 scripts/prof_driver.py > gpurun_out/rvf/fast.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/rvf/route1 -o t -- python3 scripts/prof_partitioned.py rccl1 1 $N 1 > gpurun_out/rvf/route1.log 2>&1 || exit 1
python3 - <<'PY'
import csv
def lv(path, key):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), int(r["Grid_Size_X"]) // 256) for r in rows if key in r["Kernel_Name"]]
    return d[len(d) // 2:]
f = lv("gpurun_out/rvf/fast/t_kernel_trace.csv", "expand_fast")
r = lv("gpurun_out/rvf/route1/t_kernel_trace.csv", "expand_route")
print(f"expand_fast {sum(x for x, _ in f) / 1e6:.2f} ms in {len(f)} launches; expand_route (1 partition) {sum(x for x, _ in r) / 1e6:.2f} ms in {len(r)}")
for i in range(max(len(f), len(r))):
    a = f[i] if i < len(f) else (0, 0)
    b = r[i] if i < len(r) else (0, 0)
    print(f"  {i:3d} fast {a[0] / 1e3:9.1f} us grid {a[1]:5d} | route {b[0] / 1e3:9.1f} us grid {b[1]:5d}")
PY
