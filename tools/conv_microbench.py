#!/usr/bin/env python3
"""Per-shape timing of the HIP implicit-GEMM conv kernels (fwd / dgrad / wgrad) on ResNet-50 shapes,
next to MIOpen (torch.nn.functional.conv2d, channels_last bf16) as the reference point."""
import ctypes
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_tensorflow_models_amd.ops import _lib  # noqa: E402
from distributed_tensorflow_models_amd.ops.geometry import conv_geom  # noqa: E402

B = int(os.environ.get("B", "256"))
SHAPES = [  # H, C, K, R, stride, pad, count in resnet50
    (224, 8, 64, 7, 2, 3, 1),
    (56, 64, 256, 1, 1, 0, 4), (56, 64, 64, 1, 1, 0, 1), (56, 64, 64, 3, 1, 1, 2), (56, 256, 64, 1, 1, 0, 2),
    (56, 64, 64, 3, 2, 1, 1), (28, 64, 256, 1, 1, 0, 1), (28, 256, 512, 1, 1, 0, 1), (28, 256, 128, 1, 1, 0, 1),
    (28, 128, 128, 3, 1, 1, 3), (28, 128, 512, 1, 1, 0, 3), (28, 512, 128, 1, 1, 0, 3), (28, 128, 128, 3, 2, 1, 1),
    (14, 128, 512, 1, 1, 0, 1), (14, 512, 1024, 1, 1, 0, 1), (14, 512, 256, 1, 1, 0, 1), (14, 256, 256, 3, 1, 1, 5),
    (14, 256, 1024, 1, 1, 0, 5), (14, 1024, 256, 1, 1, 0, 5), (14, 256, 256, 3, 2, 1, 1), (7, 256, 1024, 1, 1, 0, 1),
    (7, 1024, 2048, 1, 1, 0, 1), (7, 1024, 512, 1, 1, 0, 1), (7, 512, 512, 3, 1, 1, 3), (7, 512, 2048, 1, 1, 0, 3),
    (7, 2048, 512, 1, 1, 0, 2),
]


def timeit(fn, n=20):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n


def main():
    L = _lib.lib()
    s = _lib.stream_ptr()
    only = os.environ.get("ONLY")
    tot = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0, "miopen_fwd": 0.0, "miopen_bwd": 0.0}
    print("%-28s %9s %9s %9s | %9s %9s" % ("shape", "fwd", "dgrad", "wgrad", "mio_fwd", "mio_bwd"))
    for (H, C, K, R, st, pad, cnt) in SHAPES:
        if only and only not in "%d_%d_%d_%d" % (H, C, K, R):
            continue
        x = torch.randn(B, H, H, C, device="cuda").to(torch.bfloat16)
        w = (torch.randn(K, R, R, C, device="cuda") * 0.05).to(torch.bfloat16)
        g = conv_geom(tuple(x.shape), tuple(w.shape), st, (pad, pad))
        d = g.as_desc(_lib.ConvDesc)
        y = torch.empty(B, g.P, g.Q, K, device="cuda", dtype=torch.bfloat16)
        dy = torch.randn_like(y)
        wt = torch.empty(C, R, R, K, device="cuda", dtype=torch.bfloat16)
        L.dtm_weight_flip_transpose(_lib.ptr(w), _lib.ptr(wt), K, R, R, C, s)
        dx = torch.empty_like(x)
        dw = torch.zeros(K, R, R, C, device="cuda")
        fl = 2.0 * B * g.P * g.Q * K * R * R * C
        tf = timeit(lambda: L.dtm_conv_fwd(_lib.ptr(x), _lib.ptr(w), _lib.ptr(y), None, None, None, None, 0,
                                           ctypes.byref(d), s))
        td = timeit(lambda: L.dtm_conv_dgrad(_lib.ptr(dy), _lib.ptr(wt), _lib.ptr(dx), ctypes.byref(d), s))
        tw = timeit(lambda: L.dtm_conv_wgrad(_lib.ptr(x), _lib.ptr(dy), _lib.ptr(dw), None, None, ctypes.byref(d),
                                             _lib.num_cus(), s))
        mf = mb = 0.0
        if not os.environ.get("NOMIO"):
            xc = x.permute(0, 3, 1, 2)
            wc = w.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
            xg = xc.detach().requires_grad_()
            wg = wc.detach().requires_grad_()
            mf = timeit(lambda: torch.nn.functional.conv2d(xc, wc, None, st, pad))
            yy = torch.nn.functional.conv2d(xg, wg, None, st, pad)
            gy = torch.randn_like(yy)
            mb = timeit(lambda: torch.autograd.grad(torch.nn.functional.conv2d(xg, wg, None, st, pad), (xg, wg),
                                                    gy)) - mf
        for k, v in (("fwd", tf), ("dgrad", td), ("wgrad", tw), ("miopen_fwd", mf), ("miopen_bwd", mb)):
            tot[k] += v * cnt
        name = "H%d C%d K%d R%d s%d x%d" % (H, C, K, R, st, cnt)
        print("%-28s %6.0fus %4.0fT %6.0fus %4.0fT %6.0fus %4.0fT | %6.0fus %6.0fus" % (
            name, tf * 1e6, fl / tf / 1e12, td * 1e6, fl / td / 1e12, tw * 1e6, fl / tw / 1e12, mf * 1e6, mb * 1e6),
            flush=True)
    print("TOTAL per step (weighted): fwd %.2f ms  dgrad %.2f ms  wgrad %.2f ms  | miopen fwd %.2f ms bwd %.2f ms" % (
        tot["fwd"] * 1e3, tot["dgrad"] * 1e3, tot["wgrad"] * 1e3, tot["miopen_fwd"] * 1e3, tot["miopen_bwd"] * 1e3))


if __name__ == "__main__":
    main()
