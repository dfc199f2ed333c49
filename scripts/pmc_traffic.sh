#!/bin/bash
# Beyond-L2 memory traffic of the bench's expand kernel from rocprofv3 PMC counters, in separate
# passes (counters only with --kernel-trace; never with sys/runtime traces on this pool).
# Reads: TCC_EA0_RDREQ_{128B,64B,32B} x their sizes (FETCH_SIZE tallies 128-B requests at 64 B on
# gfx950, MI355X_MICROARCH.md §HBM, so the sized request counters are used directly).
# Writes: WRITE_SIZE (KiB). Atomics: TCC_EA0_ATOMIC (memory-side, counted separately).
# Infinity-Cache hits are included (they are beyond L2). Output: profiles/pmc_traffic.json.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/pmc_traffic
mkdir -p $OUT
CMD="python3 bench.py --steps 2 --warmup 1 --cpu-baseline 0 --config4-steps 0"
timeout -k 10 180 rocprofv3 --pmc TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_ATOMIC_sum --kernel-trace --output-format csv -d $OUT/a -o a -- $CMD > $OUT/a.log 2>&1
timeout -k 10 180 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/b -o b -- $CMD > $OUT/b.log 2>&1
python3 - <<'PY'
import csv, json, collections
def load(path):
    rows = list(csv.DictReader(open(path)))
    ex = [r for r in rows if "expand_fast" in r["Kernel_Name"]]
    tot = collections.defaultdict(float)
    for r in ex:
        tot[r["Counter_Name"]] += float(r["Counter_Value"])
    n = len({r["Dispatch_Id"] for r in ex})
    return tot, n
a, na = load("gpurun_out/pmc_traffic/a/a_counter_collection.csv")
b, nb = load("gpurun_out/pmc_traffic/b/b_counter_collection.csv")
rd = (a["TCC_EA0_RDREQ_128B_sum"] * 128 + a["TCC_EA0_RDREQ_64B_sum"] * 64 + a["TCC_EA0_RDREQ_32B_sum"] * 32) / na
wr = b["WRITE_SIZE"] * 1024 / nb
res = {"rm_count": 9, "n_gpus": 1, "kernel": "expand_fast<TwoPhase>", "launches": na,
       "read_bytes_per_launch": rd, "write_bytes_per_launch": wr, "bytes_per_launch": rd + wr,
       "atomics_per_launch": a["TCC_EA0_ATOMIC_sum"] / na,
       "note": "beyond-L2 (Infinity Cache + HBM) bytes from TCC_EA0_RDREQ_{128B,64B,32B} and WRITE_SIZE, "
               "averaged over every expand_fast dispatch of `bench.py --steps 2 --warmup 1` (3 full checks)"}
json.dump(res, open("profiles/pmc_traffic.json", "w"), indent=1)
json.dump(res, open("gpurun_out/pmc_traffic/pmc_traffic.json", "w"), indent=1)  # gpurun merges this one back
print(json.dumps(res))
PY
