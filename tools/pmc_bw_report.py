#!/usr/bin/env python3
"""Join the FETCH_SIZE and WRITE_SIZE passes of tools/pmc_bw.sh: per kernel name, HBM bytes and
the achieved bandwidth (bytes / kernel time).  Usage: pmc_bw_report.py FETCH_CSV WRITE_CSV STEPS [TOP]."""
import collections
import csv
import re
import sys


def load(path):
    rows = list(csv.DictReader(open(path)))
    return [(re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", ""), float(r["Counter_Value"]),
             int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) for r in rows]


def main():
    f, w, steps = load(sys.argv[1]), load(sys.argv[2]), int(sys.argv[3])
    top = int(sys.argv[4]) if len(sys.argv) > 4 else 30
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0, 0])
    n = min(len(f), len(w))
    for (name, fk, t), (name2, wk, t2) in zip(f[:n], w[:n]):
        a = agg[name[:60]]
        a[0] += 1
        a[1] += fk * 1024
        a[2] += wk * 1024
        a[3] += min(t, t2)
    tot_t = sum(a[3] for a in agg.values())
    tot_b = sum(a[1] + a[2] for a in agg.values())
    print("per step: %.2f ms kernel time, %.2f GB moved, %.2f TB/s average" % (
        tot_t / steps / 1e6, tot_b / steps / 1e9, tot_b / tot_t / 1e3))
    print("%-60s %6s %9s %9s %9s %8s" % ("kernel", "calls", "ms/step", "rd GB", "wr GB", "TB/s"))
    for name, (c, fb, wb, t) in sorted(agg.items(), key=lambda kv: -kv[1][3])[:top]:
        print("%-60s %6d %9.3f %9.3f %9.3f %8.2f" % (name, c // steps, t / steps / 1e6, fb / steps / 1e9,
                                                   wb / steps / 1e9, (fb + wb) / max(t, 1) / 1e3))


if __name__ == "__main__":
    main()
