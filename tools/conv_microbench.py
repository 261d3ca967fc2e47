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
    if os.environ.get("DEC_TILE") is not None:  # A/B: grouped strided-dgrad tile for the whole grouped grid
        L.dtm_conv_set_dec_tile(int(os.environ["DEC_TILE"]))
    if os.environ.get("DEC_LPT") is not None:  # A/B: grouped strided-dgrad classes in descending tap count
        L.dtm_conv_set_dec_lpt(int(os.environ["DEC_LPT"]))
    tot = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0, "miopen_fwd": 0.0, "miopen_bwd": 0.0, "miopen_dgrad": 0.0,
           "miopen_wgrad": 0.0}
    print("%-24s %14s %14s %14s | %14s %14s %14s | %s" % ("shape", "fwd", "dgrad", "wgrad", "mio_fwd", "mio_dgrad",
                                                           "mio_wgrad", "ours/miopen f d w"))
    for (H, C, K, R, st, pad, cnt) in SHAPES:
        if only and only not in "%d_%d_%d_%d" % (H, C, K, R):
            continue
        if os.environ.get("STRIDED") and st == 1:
            continue
        x = torch.randn(B, H, H, C, device="cuda").to(torch.bfloat16)
        w = (torch.randn(K, R, R, C, device="cuda") * 0.05).to(torch.bfloat16)
        g = conv_geom(tuple(x.shape), tuple(w.shape), st, (pad, pad))
        d = g.as_desc(_lib.ConvDesc)
        y = torch.empty(B, g.P, g.Q, K, device="cuda", dtype=torch.bfloat16)
        dy = torch.randn_like(y)
        wt = torch.empty(C, R, R, K, device="cuda", dtype=torch.bfloat16)
        if st > 1 and R >= st and not os.environ.get("NODEC"):
            # strided dgrad: the stride-decomposed form the training path uses (ConvDesc.dec)
            L.dtm_weight_flip_transpose_dec(_lib.ptr(w), _lib.ptr(wt), K, R, R, C, st, pad, pad, s)
            d.dec = 1
        else:
            L.dtm_weight_flip_transpose(_lib.ptr(w), _lib.ptr(wt), K, R, R, C, s)
        dx = torch.empty_like(x)
        dw = torch.zeros(K, R, R, C, device="cuda")
        fl = 2.0 * B * g.P * g.Q * K * R * R * C
        tf = timeit(lambda: L.dtm_conv_fwd(_lib.ptr(x), _lib.ptr(w), _lib.ptr(y), None, None, None, None, 0,
                                           ctypes.byref(d), s))
        td = timeit(lambda: L.dtm_conv_dgrad(_lib.ptr(dy), _lib.ptr(wt), _lib.ptr(dx), ctypes.byref(d), s))
        d.dec = 0
        tw = timeit(lambda: L.dtm_conv_wgrad(_lib.ptr(x), _lib.ptr(dy), _lib.ptr(dw), None, None, ctypes.byref(d),
                                             _lib.num_cus(), s))
        mf = mb = md = mw = 0.0
        if not os.environ.get("NOMIO"):
            xc = x.permute(0, 3, 1, 2)
            wc = w.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
            xg = xc.detach().requires_grad_()
            wg = wc.detach().requires_grad_()
            mf = timeit(lambda: torch.nn.functional.conv2d(xc, wc, None, st, pad))
            yy = torch.nn.functional.conv2d(xg, wg, None, st, pad)
            gy = torch.randn_like(yy)
            cb = torch.ops.aten.convolution_backward
            md = timeit(lambda: cb(gy, xc, wc, None, (st, st), (pad, pad), (1, 1), False, (0, 0), 1,
                                   (True, False, False)))
            mw = timeit(lambda: cb(gy, xc, wc, None, (st, st), (pad, pad), (1, 1), False, (0, 0), 1,
                                   (False, True, False)))
            mb = md + mw
        for k, v in (("fwd", tf), ("dgrad", td), ("wgrad", tw), ("miopen_fwd", mf), ("miopen_bwd", mb),
                     ("miopen_dgrad", md), ("miopen_wgrad", mw)):
            if H == 224 and "dgrad" in k:
                continue  # the stem's input gradient is never computed in training (the image needs none)
            tot[k] += v * cnt
        name = "H%d C%d K%d R%d s%d x%d" % (H, C, K, R, st, cnt)
        tfl = lambda t: fl / t / 1e12 if t > 0 else 0.0  # noqa: E731
        rat = lambda a, b: b / a if (a > 0 and b > 0) else 0.0  # noqa: E731
        print("%-24s %6.0fus %5.0fT %6.0fus %5.0fT %6.0fus %5.0fT | %6.0fus %5.0fT %6.0fus %5.0fT %6.0fus %5.0fT |"
              " %4.2f %4.2f %4.2f" % (
                  name, tf * 1e6, tfl(tf), td * 1e6, tfl(td), tw * 1e6, tfl(tw), mf * 1e6, tfl(mf), md * 1e6, tfl(md),
                  mw * 1e6, tfl(mw), rat(tf, mf), rat(td, md), rat(tw, mw)), flush=True)
    print("TOTAL per step (weighted, stem dgrad excluded): fwd %.2f ms  dgrad %.2f ms  wgrad %.2f ms  | miopen fwd %.2f ms dgrad %.2f ms "
          "wgrad %.2f ms" % (tot["fwd"] * 1e3, tot["dgrad"] * 1e3, tot["wgrad"] * 1e3, tot["miopen_fwd"] * 1e3,
                             tot["miopen_dgrad"] * 1e3, tot["miopen_wgrad"] * 1e3))
    print("(speed ratio columns: MIOpen time / ours; > 1 = ours faster)")


if __name__ == "__main__":
    main()
