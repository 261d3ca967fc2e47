#!/usr/bin/env python3
"""Compact per-step summary of a rocprofv3 kernel_stats.csv: python tools/prof_summary.py CSV STEPS [TOP]."""
import csv
import re
import sys


def short(name):
    name = re.sub(r"\(.*", "", name)
    name = name.replace("void ", "").replace("at::native::", "aten::")
    return name[:70]


def main():
    path, steps = sys.argv[1], int(sys.argv[2])
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
    rows = list(csv.DictReader(open(path)))
    tot = sum(int(r["TotalDurationNs"]) for r in rows)
    print("total GPU time per step: %.2f ms" % (tot / steps / 1e6))
    for r in rows[:top]:
        t = int(r["TotalDurationNs"])
        print("%8.3f ms/step %5.1f%%  %5d calls  avg %8.1f us  %s" % (
            t / steps / 1e6, 100.0 * t / tot, int(r["Calls"]) // steps, float(r["AverageNs"]) / 1e3, short(r["Name"])))


if __name__ == "__main__":
    main()
