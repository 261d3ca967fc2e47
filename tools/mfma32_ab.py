#!/usr/bin/env python3
"""Per-shape same-process A/B of the conv kernels' MFMA shape (16x16x32 vs the 32x32x16 forms of the
LDS-DMA tiles, dtm_conv_set_mfma32) on the ResNet-50 shapes (fwd with BN statistics, dgrad), interleaved
repetitions, plus the max difference of the two outputs (fp32 summation order only).
Usage: python tools/mfma32_ab.py  (B=256)"""
import ctypes
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_tensorflow_models_amd.ops import _lib  # noqa: E402
from distributed_tensorflow_models_amd.ops.geometry import conv_geom  # noqa: E402
from tools.conv_microbench import SHAPES  # noqa: E402

B = int(os.environ.get("B", "256"))


def timed(fn, n=10):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e6


def main():
    L = _lib.lib()
    s = _lib.stream_ptr()
    tot = {0: 0.0, 1: 0.0}
    print("%-26s %-6s %9s %9s %7s %9s" % ("shape", "pass", "mfma16", "mfma32", "gain", "maxdiff"))
    for (H, C, K, R, st, pad, cnt) in SHAPES:
        if H == 224:
            continue
        x = torch.randn(B, H, H, C, device="cuda").to(torch.bfloat16)
        w = (torch.randn(K, R, R, C, device="cuda") * 0.05).to(torch.bfloat16)
        g = conv_geom(tuple(x.shape), tuple(w.shape), st, (pad, pad))
        d = g.as_desc(_lib.ConvDesc)
        y = [torch.empty(B, g.P, g.Q, K, device="cuda", dtype=torch.bfloat16) for _ in range(2)]
        stats = torch.zeros(2, K, device="cuda")
        dy = torch.randn_like(y[0])
        wt = torch.empty(C, R, R, K, device="cuda", dtype=torch.bfloat16)
        dec = st > 1 and R >= st
        if dec:
            L.dtm_weight_flip_transpose_dec(_lib.ptr(w), _lib.ptr(wt), K, R, R, C, st, pad, pad, s)
        else:
            L.dtm_weight_flip_transpose(_lib.ptr(w), _lib.ptr(wt), K, R, R, C, s)
        dx = [torch.empty_like(x) for _ in range(2)]

        def fwd(v):
            L.dtm_conv_set_mfma32(v)
            L.dtm_conv_fwd(_lib.ptr(x), _lib.ptr(w), _lib.ptr(y[v]), _lib.ptr(stats), None, None, None, 0,
                           ctypes.byref(d), s)

        def dgr(v):
            L.dtm_conv_set_mfma32(v)
            d.dec = int(dec)
            L.dtm_conv_dgrad(_lib.ptr(dy), _lib.ptr(wt), _lib.ptr(dx[v]), ctypes.byref(d), s)
            d.dec = 0

        for name, fn, out in (("fwd", fwd, y), ("dgrad", dgr, dx)):
            for v in (0, 1):
                fn(v)
            res = {0: [], 1: []}
            for _ in range(5):
                for v in (0, 1):
                    res[v].append(timed(lambda: fn(v)))
            m = {v: statistics.median(res[v]) for v in (0, 1)}
            diff = ((out[0].float() - out[1].float()).abs().max() / (out[0].float().abs().max() + 1e-9)).item()
            for v in (0, 1):
                tot[v] += m[v] * cnt
            print("H%-3d C%-4d K%-4d R%d s%d x%d  %-6s %8.1fus %8.1fus %+6.1f%% %9.2e" % (
                H, C, K, R, st, cnt, name, m[0], m[1], (m[0] / m[1] - 1) * 100, diff), flush=True)
    L.dtm_conv_set_mfma32(0)
    print("TOTAL fwd+dgrad per step (weighted): mfma16 %.3f ms  mfma32 %.3f ms  (%+.1f %%)" % (
        tot[0] / 1e3, tot[1] / 1e3, (tot[0] / tot[1] - 1) * 100))


if __name__ == "__main__":
    main()
