#!/usr/bin/env python3
"""Timing of the merged sibling-head forward (dtm_conv_fwd_bn_multi: one 1x1 conv over the concatenated head weights,
split epilogue, grouped BN finalize) on the Inception-v3 mixed-block head shapes (batch 128), for the tile the
shape policy picks or a forced one (DTM_CONV_TILE, read once per process: run one process per tile).

  DTM_CONV_TILE=21 python tools/split_tile_sweep.py
"""
import ctypes
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_tensorflow_models_amd.ops import _lib  # noqa: E402

B = int(os.environ.get("B", "128"))
# (H, C, member widths, blocks of this shape per step)
SHAPES = [(35, 192, (64, 48, 64, 32), 1), (35, 256, (64, 48, 64, 64), 1), (35, 288, (64, 48, 64, 64), 1),
          (17, 768, (192, 128, 128, 192), 1), (17, 768, (192, 160, 160, 192), 2), (17, 768, (192, 192, 192, 192), 1),
          (17, 768, (192, 192), 1), (8, 1280, (320, 384, 448, 192), 1), (8, 2048, (320, 384, 448, 192), 1)]


def main():
    L = _lib.lib()
    s = _lib.stream_ptr()
    tot = 0.0
    for H, C, ks, cnt in SHAPES:
        Kt = sum(ks)
        x = torch.randn(B, H, H, C, device="cuda").to(torch.bfloat16)
        w = (torch.randn(Kt, 1, 1, C, device="cuda") * 0.05).to(torch.bfloat16)
        ys = [torch.empty(B, H, H, k, device="cuda", dtype=torch.bfloat16) for k in ks]
        bn = []
        keep = []
        for k in ks:
            t = [torch.ones(k, device="cuda"), torch.zeros(k, device="cuda"), torch.zeros(k, device="cuda"),
                 torch.ones(k, device="cuda"), torch.empty(4, k, device="cuda")]
            keep += t
            bn += [q.data_ptr() for q in t]
        d = _lib.ConvDesc(B, H, H, C, Kt, 1, 1, H, H, 1, 0, 0, 0, 0)
        yp = (ctypes.c_void_p * len(ys))(*[y.data_ptr() for y in ys])
        kp = (ctypes.c_int * len(ks))(*ks)
        bp = (ctypes.c_void_p * len(bn))(*bn)

        def run():
            rc = L.dtm_conv_fwd_bn_multi(_lib.ptr(x), _lib.ptr(w), yp, kp, len(ks), bp, float(B * H * H), 1e-3, 0.9997,
                                         1, 0, ctypes.byref(d), s)
            assert rc == 0, rc
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        n = 30
        t0 = time.perf_counter()
        for _ in range(n):
            run()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / n
        tot += dt * cnt
        fl = 2.0 * B * H * H * Kt * C
        print("H%-3d C%-5d K%-5d (%s) x%d  %7.1f us  %5.0f TF/s" % (H, C, Kt, "+".join(map(str, ks)), cnt, dt * 1e6,
                                                                  fl / dt / 1e12), flush=True)
    print("TOTAL per step (weighted): %.1f us" % (tot * 1e6), flush=True)


if __name__ == "__main__":
    main()
