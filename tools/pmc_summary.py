#!/usr/bin/env python3
"""Per-kernel averages of a rocprofv3 --pmc counter_collection.csv (one row per dispatch and counter)."""
import collections
import csv
import re
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in rows:
        name = re.sub(r"\(.*", "", r.get("Kernel_Name", r.get("Kernel-Name", "?")))[:70]
        if r.get("Grid_Size"):  # one entry per kernel and launch shape
            name += "  grid=%s" % r["Grid_Size"]
        agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for name, cs in agg.items():
        if "conv" not in name and "wgrad" not in name:
            continue
        avg = {k: sum(v) / len(v) for k, v in cs.items()}
        wc = avg.get("SQ_WAVE_CYCLES", 0) or 1
        print(name)
        print("   " + "  ".join("%s=%.3g" % (k, v) for k, v in sorted(avg.items())))
        print("   wait_any %.0f%%  wait_inst %.0f%%  active %.0f%%  lds_inst_wait %.0f%%  bank_conflict/wave_cycle %.3f" % (
            100 * avg.get("SQ_WAIT_ANY", 0) / wc, 100 * avg.get("SQ_WAIT_INST_ANY", 0) / wc,
            100 * avg.get("SQ_ACTIVE_INST_ANY", 0) / wc, 100 * avg.get("SQ_WAIT_INST_LDS", 0) / wc,
            avg.get("SQ_LDS_BANK_CONFLICT", 0) / wc))
        if "SQ_VALU_MFMA_BUSY_CYCLES" in avg and "SQ_BUSY_CYCLES" in avg:
            # MFMA busy cycles per SIMD vs the busy time of the shader engines (1 SQ per CU: 4 SIMDs)
            print("   mfma busy / (4 x SQ busy) = %.0f%%" % (100 * avg["SQ_VALU_MFMA_BUSY_CYCLES"] /
                                                         max(1.0, 4 * avg["SQ_BUSY_CYCLES"])))


if __name__ == "__main__":
    main()
