#!/usr/bin/env python3
"""Stem max-pool kernels (BN-apply + ReLU fused, 3x3 / stride 2) at the ResNet-50 and Inception-v3 training shapes:
time and effective HBM bandwidth of the forward and backward, specialised k3s2 kernels vs the generic gather
kernels, interleaved in one process (median of ROUNDS).  Usage: python tools/pool_bench.py"""
import ctypes
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_tensorflow_models_amd.ops import _lib  # noqa: E402
from distributed_tensorflow_models_amd.ops.geometry import pool_geom  # noqa: E402

SHAPES = [("resnet50 pool1", 256, 112, 64, "SAME"), ("inception pool1", 128, 147, 64, "VALID"),
          ("inception pool2", 128, 71, 192, "VALID")]
ROUNDS = int(os.environ.get("ROUNDS", "5"))


def timed(fn, n=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


def main():
    L = _lib.lib()
    st = _lib.stream_ptr()
    for name, N, H, C, pad in SHAPES:
        raw = torch.randn(N, H, H, C, device="cuda").to(torch.bfloat16)
        ss = torch.stack([torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.3,
                          torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")]).contiguous()
        g = pool_geom(tuple(raw.shape), 3, 2, pad)
        a = g.as_args(_lib.PoolArgs)
        y = torch.empty(N, g.P, g.Q, C, device="cuda", dtype=torch.bfloat16)
        arg = torch.empty(N, g.P, g.Q, C, device="cuda", dtype=torch.uint8)
        dy = torch.randn_like(y)
        dx = torch.empty_like(raw)
        sums = torch.zeros(4, C, device="cuda")
        fwd = lambda: L.dtm_maxpool_bnrelu_fwd(_lib.ptr(raw), _lib.ptr(ss), _lib.ptr(y), _lib.ptr(arg),  # noqa
                                               ctypes.byref(a), st)
        bwd = lambda: L.dtm_maxpool_bnrelu_bwd(_lib.ptr(dy), _lib.ptr(arg), _lib.ptr(raw), _lib.ptr(ss),  # noqa
                                               _lib.ptr(dx), _lib.ptr(sums), ctypes.byref(a), 0, st)
        bx, by = raw.numel() * 2, y.numel() * 2
        bytes_ = {"fwd": bx + by + y.numel(), "bwd": by + y.numel() + 2 * bx}  # (compulsory HBM traffic)
        for pname, fn in (("fwd", fwd), ("bwd", bwd)):
            res = {0: [], 1: []}
            for _ in range(ROUNDS):
                for fast in (0, 1):
                    L.dtm_pool_set_k3s2(fast)
                    res[fast].append(timed(fn))
            L.dtm_pool_set_k3s2(1)
            m = {k: statistics.median(v) for k, v in res.items()}
            print("%-16s %s  generic %7.1f us (%4.2f TB/s)  k3s2 %7.1f us (%4.2f TB/s)  %+.1f %%" % (
                name, pname, m[0], bytes_[pname] / m[0] / 1e6, m[1], bytes_[pname] / m[1] / 1e6,
                100.0 * (m[1] - m[0]) / m[0]), flush=True)


def avg_main():
    """3x3 / stride-1 SAME average pools of Inception-v3's pool branches (batch 128)."""
    L = _lib.lib()
    st = _lib.stream_ptr()
    for name, N, H, C in (("inc 35x35x64", 128, 35, 64), ("inc 35x35x32", 128, 35, 32), ("inc 17x17x192", 128, 17, 192),
                          ("inc 8x8x192", 128, 8, 192)):
        x = torch.randn(N, H, H, C, device="cuda").to(torch.bfloat16)
        g = pool_geom(tuple(x.shape), 3, 1, "SAME")
        a = g.as_args(_lib.PoolArgs)
        y = torch.empty_like(x)
        dy, dx = torch.randn_like(x), torch.empty_like(x)
        fwd = lambda: L.dtm_avgpool_fwd(_lib.ptr(x), _lib.ptr(y), ctypes.byref(a), 0, st)  # noqa
        bwd = lambda: L.dtm_avgpool_bwd(_lib.ptr(dy), _lib.ptr(dx), ctypes.byref(a), 0, st)  # noqa
        for pname, fn in (("fwd", fwd), ("bwd", bwd)):
            res = {0: [], 1: []}
            for _ in range(ROUNDS):
                for fast in (0, 1):
                    L.dtm_pool_set_k3s2(fast)
                    res[fast].append(timed(fn))
            L.dtm_pool_set_k3s2(1)
            m = {k: statistics.median(v) for k, v in res.items()}
            b = 2 * x.numel() * 2
            print("%-16s %s  generic %7.1f us (%4.2f TB/s)  k3s1 %7.1f us (%4.2f TB/s)  %+.1f %%" % (
                name, pname, m[0], b / m[0] / 1e6, m[1], b / m[1] / 1e6, 100.0 * (m[1] - m[0]) / m[0]), flush=True)


def cat_main():
    """One-launch zero-copy concat of BN'd branch outputs (dtm_cat_bn_apply / _bwd) at Inception-v3's mixed-block
    widths (batch 128); compare two library builds with DTM_KERNELS_SO."""
    from distributed_tensorflow_models_amd.ops.fused import _ConcatBNApplyFn as _ConcatFn
    L = _lib.lib()
    st = _lib.stream_ptr()
    for name, N, H, Cs in (("cat 35x35x288", 128, 35, (64, 64, 96, 64)), ("cat 17x17x768", 128, 17, (192,) * 4),
                           ("cat 8x8x1280", 128, 8, (320, 384, 384, 192)), ("cat 8x8x2048", 128, 8, (320, 768, 768, 192))):
        M, Ct = N * H * H, sum(Cs)
        raws = [torch.randn(M, c, device="cuda").to(torch.bfloat16) for c in Cs]
        sss = [torch.stack([torch.rand(c, device="cuda") + 0.5, torch.randn(c, device="cuda") * 0.3,
                            torch.zeros(c, device="cuda"), torch.ones(c, device="cuda")]) for c in Cs]
        masks = [torch.empty(M * c // 8, device="cuda", dtype=torch.uint8) for c in Cs]
        dxs = [torch.empty_like(r) for r in raws]
        tab = _ConcatFn._descs([(r, ss, m, dx, c, 1) for r, ss, m, dx, c in zip(raws, sss, masks, dxs, Cs)])
        out = torch.empty(M, Ct, device="cuda", dtype=torch.bfloat16)
        dout = torch.randn_like(out)
        sums = torch.zeros(4 * Ct, device="cuda")
        fwd = lambda: L.dtm_cat_bn_apply(ctypes.c_void_p(tab.ctypes.data), len(Cs), _lib.ptr(out), M, Ct, st)  # noqa
        bwd = lambda: L.dtm_cat_bn_apply_bwd(ctypes.c_void_p(tab.ctypes.data), len(Cs), _lib.ptr(dout),  # noqa
                                             _lib.ptr(sums), M, Ct, st)
        b = M * Ct * 2
        for pname, fn, nbytes in (("fwd", fwd, 2 * b + M * Ct // 8), ("bwd", bwd, 3 * b + M * Ct // 8)):
            v = statistics.median([timed(fn) for _ in range(ROUNDS)])
            print("%-16s %s %7.1f us (%4.2f TB/s)" % (name, pname, v, nbytes / v / 1e6), flush=True)


if __name__ == "__main__":
    if os.environ.get("CAT"):
        cat_main()
        sys.exit(0)
    if os.environ.get("AVG"):
        avg_main()
        sys.exit(0)
    main()
