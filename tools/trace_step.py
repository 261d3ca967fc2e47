#!/usr/bin/env python3
"""One training step from a rocprofv3 kernel trace: every dispatch in order with its duration, grid
and the idle gap before it; per-kernel-name totals.  Step = dispatches after the second-to-last
optimizer launch (multi_tensor_opt_kernel) up to and including the last one.
Usage: python tools/trace_step.py gpurun_out/prof/run_kernel_trace.csv [--top N]"""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 40
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    opt = [i for i, r in enumerate(rows) if "multi_tensor_opt" in r["Kernel_Name"]]
    lo, hi = opt[-2] + 1, opt[-1] + 1
    step = rows[lo:hi]
    t0 = int(step[0]["Start_Timestamp"])
    t1 = int(step[-1]["End_Timestamp"])
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in step)
    print("step: %d dispatches, wall %.3f ms, kernel busy %.3f ms" % (len(step), (t1 - t0) / 1e6, busy / 1e6))
    per = defaultdict(float)
    prev_end = int(rows[lo - 1]["End_Timestamp"])
    lst = []
    for r in step:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")[:60]
        per[name] += (e - s) / 1e3
        lst.append(((e - s) / 1e3, (s - prev_end) / 1e3, name, r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"],
                    r["Workgroup_Size_X"]))
        prev_end = e
    print("%-62s %9s" % ("kernel", "us/step"))
    for n, v in sorted(per.items(), key=lambda kv: -kv[1]):
        print("%-62s %9.1f" % (n, v))
    print("\nlongest dispatches:")
    for d in sorted(lst, key=lambda t: -t[0])[:top]:
        print("%8.1f us  gap %6.1f  %-60s grid %s,%s,%s wg %s" % d)
    print("\ntotal idle gaps %.1f us" % sum(max(0.0, d[1]) for d in lst))


if __name__ == "__main__":
    main()
