#!/usr/bin/env python3
"""Per-kernel HBM-bytes / FLOP roofline table of ONE training step from rocprofv3 counter passes
(tools/gpu_runs/gpu_r5_*.sh: each pass `rocprofv3 --pmc <counters> --kernel-trace --output-format csv` over a short
bench.py run).  Passes are joined per dispatch (Dispatch_Id; every pass runs the same deterministic launch
sequence), the step is delimited by the fused optimizer launch (multi_tensor_opt_kernel ends every step) and the
last STEPS steps are averaged.  Under counter collection the kernels run serialized, so each kernel's duration is
its own (no side-stream overlap): the table is per-kernel cost, not the overlapped step wall time.

Byte counters (whichever the passes hold):
  rd: TCC_EA0_RDREQ_{32B,64B,128B}_sum x {32,64,128} B if present, else FETCH_SIZE (KiB; on gfx950 it books a
      128-B streaming read as 64 B - MI355X_MICROARCH.md - so it undercounts wide reads up to 2x)
  wr: WRITE_SIZE (KiB)
  flops: SQ_INSTS_VALU_MFMA_MOPS_BF16 x 512
Bounds: HBM 8.0 TB/s, bf16 dense MFMA 2.5 PF/s; floor = max(bytes / HBM, flops / MFMA); eff = floor / time.
Both rd and wr count L2 <-> fabric traffic, which Infinity-Cache (MALL) hits also pass through.

Usage: roofline_report.py STEPS CSV [CSV ...] [--top N]"""
import collections
import csv
import re
import sys

HBM_TBS, MFMA_PFS = 8.0, 2.5


def load(path):
    """Dispatch_Id -> (name, ns, {counter: value})"""
    out = {}
    for r in csv.DictReader(open(path)):
        d = int(r["Dispatch_Id"])
        name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").strip()
        e = out.setdefault(d, [name, int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), {}])
        e[1] = min(e[1], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        e[2][r["Counter_Name"]] = e[2].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return out


def main():
    args = sys.argv[1:]
    top = 40
    if "--top" in args:
        i = args.index("--top")
        top = int(args[i + 1])
        del args[i:i + 2]
    steps, paths = int(args[0]), args[1:]
    passes = [load(p) for p in paths]
    ids = sorted(set.intersection(*[set(p) for p in passes]))
    disp = []
    for d in ids:
        name, ns, ctr = passes[0][d][0], min(p[d][1] for p in passes), {}
        for p in passes:
            assert p[d][0] == name, "passes disagree at dispatch %d: %s vs %s" % (d, name, p[d][0])
            ctr.update(p[d][2])
        disp.append((name, ns, ctr))
    ends = [i for i, (n, _t, _c) in enumerate(disp) if "multi_tensor_opt_kernel" in n]
    assert len(ends) > steps, "only %d optimizer launches for %d steps" % (len(ends), steps)
    window = disp[ends[-steps - 1] + 1:ends[-1] + 1]

    def rd_bytes(c):
        if "TCC_EA0_RDREQ_128B_sum" in c:
            return (c.get("TCC_EA0_RDREQ_32B_sum", 0) * 32 + c.get("TCC_EA0_RDREQ_64B_sum", 0) * 64 +
                    c["TCC_EA0_RDREQ_128B_sum"] * 128)
        return c.get("FETCH_SIZE", 0.0) * 1024
    agg = collections.OrderedDict()
    for name, ns, c in window:
        a = agg.setdefault(name, [0, 0.0, 0.0, 0.0, 0.0])
        a[0] += 1
        a[1] += ns
        a[2] += rd_bytes(c)
        a[3] += c.get("WRITE_SIZE", 0.0) * 1024
        a[4] += c.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0.0) * 512
    src = "TCC_EA0_RDREQ_*B" if any("TCC_EA0_RDREQ_128B_sum" in c for _n, _t, c in window) else "FETCH_SIZE"
    have_fl = any("SQ_INSTS_VALU_MFMA_MOPS_BF16" in c for _n, _t, c in window)
    T = sum(a[1] for a in agg.values()) / steps
    R = sum(a[2] for a in agg.values()) / steps
    W = sum(a[3] for a in agg.values()) / steps
    FL = sum(a[4] for a in agg.values()) / steps
    print("one step (mean of the last %d; rd from %s): %d launches, %.3f ms serialized kernel time, %.2f GB read + "
          "%.2f GB written = %.2f GB (%.2f TB/s average)%s" % (
              steps, src, len(window) // steps, T / 1e6, R / 1e9, W / 1e9, (R + W) / 1e9, (R + W) / max(T, 1) / 1e3,
              ", %.3f TFLOP bf16 MFMA (%.0f TF/s)" % (FL / 1e12, FL / max(T, 1) / 1e3) if have_fl else ""))
    floor_total = 0.0
    rows = []
    for name, (n, ns, rb, wb, fl) in agg.items():
        t = ns / steps
        byt = (rb + wb) / steps
        f = fl / steps
        floor = max(byt / (HBM_TBS * 1e3), f / (MFMA_PFS * 1e6))  # ns
        floor_total += floor
        bound = "MFMA" if f / (MFMA_PFS * 1e6) > byt / (HBM_TBS * 1e3) else "HBM"
        rows.append((t, name, n // steps, byt, f, floor, bound))
    rows.sort(reverse=True)
    print("sum of per-kernel roofline floors %.3f ms = %.0f %% of the serialized kernel time" % (
        floor_total / 1e6, 100 * floor_total / max(T, 1)))
    print("%-70s %5s %8s %6s %8s %7s %7s %5s %5s" % ("kernel", "calls", "ms/step", "%time", "GB/step", "TB/s",
                                                      "TF/s", "bound", "eff%"))
    for t, name, n, byt, f, floor, bound in rows[:top]:
        print("%-70s %5d %8.3f %6.1f %8.3f %7.2f %7.0f %5s %5.0f" % (
            name[:70], n, t / 1e6, 100 * t / T, byt / 1e9, byt / max(t, 1) / 1e3, f / max(t, 1) / 1e3 if have_fl else 0,
            bound, 100 * floor / max(t, 1)))
    rest = rows[top:]
    if rest:
        print("%-70s %5d %8.3f %6.1f %8.3f" % ("(%d more kernels)" % len(rest), sum(r[2] for r in rest),
                                             sum(r[0] for r in rest) / 1e6, 100 * sum(r[0] for r in rest) / T,
                                             sum(r[3] for r in rest) / 1e9))


if __name__ == "__main__":
    main()
