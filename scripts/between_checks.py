"""What the GPU does between two back-to-back checks, from a rocprofv3 kernel trace of bench.py
(scripts/ktrace.sh): for a few consecutive checks, the launches from the last level launch of one
check to the second level launch of the next (times relative to the end of that last level
launch), and the span from one check's first launch to the next one's.

    python scripts/between_checks.py gpurun_out/<dir>/trace_kernel_trace.csv [label]
"""
import csv
import sys


def main(path, label=""):
    rows = list(csv.DictReader(open(path)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    starts = [i for i, e in enumerate(ev) if "roots_" in e[2]]
    print(f"# {label} {path}: {len(starts)} checks")
    for s in starts[6:8]:
        j = s - 1
        while "expand" not in ev[j][2]:
            j -= 1
        t0 = ev[j][1]
        k = s + 1
        while "expand" not in ev[k][2]:
            k += 1
        for e in ev[j:k + 2]:
            name = e[2].split("(")[0].replace("void ", "")[:48]
            print(f"  {(e[0] - t0) / 1e3:8.1f} .. {(e[1] - t0) / 1e3:8.1f} us  {name}")
        print()
    # the bench's timed checks: after --warmup 2, the next 10 (later ones are its profiled passes)
    spans = sorted((ev[b][0] - ev[a][0]) / 1e3 for a, b in zip(starts[2:11], starts[3:12]))
    print(f"  check span of the timed checks (first launch to the next check's), median of {len(spans)}: "
          f"{spans[len(spans) // 2]:.1f} us\n")


if __name__ == "__main__":
    main(*sys.argv[1:])
