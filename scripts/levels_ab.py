"""Per-level kernel time of gpu_env_ab.sh runs: the median over repetitions of each level's
expand launch (bench.py `levels.kernel_us`, the HIP-event pass), one column per environment.
    python3 scripts/levels_ab.py gpurun_out/<tag> "<env A>" "<env B>" ...
"""
import glob
import json
import statistics
import sys

d = sys.argv[1]
envs = sys.argv[2:]
cols, fronts, totals, probes = [], None, [], {}
for i, _ in enumerate(envs):
    runs = []
    ms = []
    for f in sorted(glob.glob(f"{d}/e{i}_r*.json")):
        line = json.loads(open(f).read().strip().splitlines()[-1])
        runs.append(line["levels"]["kernel_us"])
        ms.append(line["ms_per_step"])
        probes.setdefault(i, []).append((line.get("roofline") or {}).get("probes_per_step"))
        fronts = line["levels"].get("frontier", fronts)
    n = min(len(r) for r in runs)
    cols.append([statistics.median(r[k] for r in runs) for k in range(n)])
    totals.append(ms)
print("level frontier " + " ".join(f"{'e%d' % i:>7}" for i in range(len(envs))) + "   best")
for k in range(max(len(c) for c in cols)):
    vals = [c[k] if k < len(c) else float("nan") for c in cols]
    best = min(range(len(vals)), key=lambda i: vals[i])
    fr = fronts[k] if fronts and k < len(fronts) else ""
    print(f"{k:5d} {fr:>8} " + " ".join(f"{v:7.1f}" for v in vals) + f"   e{best}")
for i, e in enumerate(envs):
    print(f"e{i} [{e}] ms per check: " + " ".join(f"{x:.4f}" for x in totals[i]) + f"  kernel sum {sum(cols[i]):.1f} us  probes/check {probes.get(i)}")
