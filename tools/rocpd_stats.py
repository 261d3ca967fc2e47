#!/usr/bin/env python3
"""Per-kernel statistics from a rocprofv3 rocpd database (the default output format, ``run_results.db``): the same
columns as rocprofv3's ``--stats`` kernel_stats.csv (name, calls, total / average / min / max ns, percentage).

Usage: python tools/rocpd_stats.py RUN_RESULTS.db [-o kernel_stats.csv]"""
import argparse
import csv
import sqlite3
import sys


def stats(db):
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, count(*), sum(duration), min(duration), max(duration) from kernels "
                          "group by name order by sum(duration) desc"))
    total = sum(r[2] for r in rows) or 1
    return [(n, k, s, s / k, 100.0 * s / total, lo, hi) for n, k, s, lo, hi in rows]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("-o", "--out")
    a = ap.parse_args()
    out = open(a.out, "w", newline="") if a.out else sys.stdout
    w = csv.writer(out, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for r in stats(a.db):
        w.writerow([r[0], r[1], r[2], round(r[3], 1), round(r[4], 2), r[5], r[6]])


if __name__ == "__main__":
    main()
