#!/usr/bin/env python3
"""Kernel sequence of ONE training step from a rocprofv3 kernel trace (bench.py run): the last step is
the span from the last multi_tensor_opt_kernel's predecessor step boundary.  Prints each dispatch
with its duration, grid, and the idle gap before it, so per-layer costs can be read in order.
Usage: step_timeline.py run_kernel_trace.csv [--short]"""
import csv
import re
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    opt = [i for i, r in enumerate(rows) if "multi_tensor_opt" in r["Kernel_Name"]]
    if len(opt) < 2:
        sys.exit("need >= 2 steps in the trace")
    a, b = opt[-2] + 1, opt[-1] + 1
    tot = 0.0
    per_stream = {}
    prev_end = int(rows[a - 1]["End_Timestamp"])
    for r in rows[a:b]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("dtm::", "")
        d = (e - s) / 1e3
        tot += d
        sid = r.get("Stream_Id", "0")
        per_stream[sid] = per_stream.get(sid, 0.0) + d
        grid = "%sx%s" % (int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]), r["Grid_Size_Y"])
        # gap: idle time since the latest end of any earlier dispatch (negative = overlapped)
        print("%8.1f us  gap %6.1f  s%-3s %-9s %s" % (d, (s - prev_end) / 1e3, sid, grid, name[:90]))
        prev_end = max(prev_end, e)
    span = (int(rows[b - 1]["End_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e3
    print("kernels %d, busy %.1f us, span %.1f us; per stream: %s" % (
        b - a, tot, span, ", ".join("s%s %.1f us" % kv for kv in sorted(per_stream.items()))))


if __name__ == "__main__":
    main()
