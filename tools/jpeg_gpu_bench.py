#!/usr/bin/env python3
"""Device JPEG decode throughput (data/jpeg.py decode paths) on a batch of ImageNet-like synthetic JPEGs (the
generator of tools/decode_cpu_cost.py: 300-500 px sides, quality 90, ~70 KB).

  host  : marker parse + unstuffing per image (dtm_jpeg_scan, one core) - the whole host share of the full device
          decode
  device: jpeg_huff_kernel (entropy decode, one workgroup per image) + jpeg_idct_kernel + jpeg_color_kernel per
          batch, timed with HIP events; the fixed-point pass histogram of the batch

Usage: python tools/jpeg_gpu_bench.py [--images 128] [--reps 10]"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", type=int, default=128)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--min-bits", type=int, default=0)
    ap.add_argument("--cfg", nargs="+", default=["256x11"], help="threads-per-image x lookup-bits variants")
    a = ap.parse_args()
    import torch

    from distributed_tensorflow_models_amd.data import jpeg
    from distributed_tensorflow_models_amd.ops import _lib
    from tools.decode_cpu_cost import make_jpegs
    jp = make_jpegs(a.images)
    st = np.empty(1 << 22, np.uint8)
    sg = np.empty(1 << 16, np.int32)
    jpeg.scan_prep(jp[0], st, sg)
    best = None
    for _ in range(3):
        t = time.process_time()
        for j in jp:
            jpeg.scan_prep(j, st, sg)
        dt = (time.process_time() - t) / len(jp) * 1e6
        best = dt if best is None else min(best, dt)
    hb = None
    for _ in range(3):
        t = time.process_time()
        for j in jp:
            jpeg.huffman_decode(j)
        dt = (time.process_time() - t) / len(jp) * 1e6
        hb = dt if hb is None else min(hb, dt)
    print("%d JPEGs, avg %.0f KB; host per image: scan prep %.1f us (host Huffman decode %.1f us)" % (
        len(jp), sum(map(len, jp)) / len(jp) / 1024.0, best, hb))
    dev = torch.device("cuda", 0)
    from distributed_tensorflow_models_amd.ops import _lib
    for cfg in a.cfg:
        nt, lk = (int(x) for x in cfg.split("x"))
        _lib.lib().dtm_jpeg_set_huff(nt, lk)
        print("-- %d threads per image, %d-bit lookup" % (nt, lk))
        run(jp, dev, a)


def run(jp, dev, a):
    import torch

    from distributed_tensorflow_models_amd.data import jpeg
    from distributed_tensorflow_models_amd.ops import _lib
    r = jpeg.decode_batch_gpu_full(jp, dev, min_bits=a.min_bits)
    torch.cuda.synchronize()
    stt = r[2].cpu().numpy()
    print("status (fixed-point passes) histogram: %s" % (
        {int(k): int(v) for k, v in zip(*np.unique(stt, return_counts=True))}))
    # time the device stages alone on the uploaded batch
    L = _lib.lib()
    preps = [jpeg.scan_prep(d) for d in jp]
    d, ncoef, nplane, nrgb, maxb, maxp = jpeg.batch_table([p[0] for p in preps])
    h, nbytes, nseg = jpeg.huff_batch_table([p[1:] for p in preps], d, a.min_bits)
    hv = np.zeros(max(nbytes, 16), np.uint8)
    for (inf, sc, s, g), hd in zip(preps, h):
        hv[int(hd["stream_off"]):int(hd["stream_off"]) + s.size] = s
    ds = torch.from_numpy(hv).to(dev)
    dseg = torch.zeros(max(nseg, 1), dtype=torch.int32, device=dev)
    dh = torch.from_numpy(h.view(np.uint8)).to(dev)
    dd = torch.from_numpy(d.view(np.uint8)).to(dev)
    coefs = torch.empty(max(ncoef, 8), dtype=torch.int16, device=dev)
    status = torch.empty(len(jp), dtype=torch.int32, device=dev)
    planes = torch.empty(max(nplane, 8), dtype=torch.uint8, device=dev)
    rgb = torch.empty(max(nrgb, 1), dtype=torch.uint8, device=dev)
    sp = _lib.stream_ptr()

    def huff():
        L.dtm_jpeg_huff_gpu(_lib.ptr(ds), _lib.ptr(dseg), _lib.ptr(dh), len(jp), _lib.ptr(coefs), _lib.ptr(status), sp)

    def rest():
        L.dtm_jpeg_decode_gpu(_lib.ptr(coefs), _lib.ptr(dd), len(jp), int(maxb), int(maxp), _lib.ptr(planes),
                              _lib.ptr(rgb), sp)
    for name, fn in (("entropy decode", huff), ("idct + colour", rest)):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.reps
        print("device %-15s: %.3f ms per batch of %d -> %.0f img/s (whole GPU)" % (name, ms, len(jp),
                                                                                  len(jp) / ms * 1e3))


if __name__ == "__main__":
    main()
