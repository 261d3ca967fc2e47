#!/usr/bin/env python3
"""A few representative conv launches, repeated, for per-kernel hardware counters (rocprofv3 --pmc ... -- python3
tools/conv_pmc_run.py; summarise with tools/pmc_summary.py).  Shapes: ResNet-50 batch 256 (14x14 3x3 256, 28x28
3x3 128, 7x7 3x3 512, 14x14 1x1 1024->256) and Inception-v3 batch 128 (17x17 1x7 160, 35x35 1x1 288->64)."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_tensorflow_models_amd.ops import _lib  # noqa: E402
from distributed_tensorflow_models_amd.ops.geometry import conv_geom  # noqa: E402

# N, H, W, C, K, R, S, stride, pad
SHAPES = [
    (256, 14, 14, 256, 256, 3, 3, 1, "SAME"),
    (256, 28, 28, 128, 128, 3, 3, 1, "SAME"),
    (256, 7, 7, 512, 512, 3, 3, 1, "SAME"),
    (256, 14, 14, 1024, 256, 1, 1, 1, "SAME"),
    (128, 17, 17, 160, 160, 1, 7, 1, "SAME"),
    (128, 35, 35, 288, 64, 1, 1, 1, "SAME"),
]


def main():
    L = _lib.lib()
    st = _lib.stream_ptr()
    reps = int(os.environ.get("REPS", "10"))
    for (N, H, W, C, K, R, S, s, pad) in SHAPES:
        x = torch.randn(N, H, W, C, device="cuda").to(torch.bfloat16)
        w = (torch.randn(K, R, S, C, device="cuda") * 0.05).to(torch.bfloat16)
        g = conv_geom(tuple(x.shape), tuple(w.shape), s, pad)
        d = g.as_desc(_lib.ConvDesc)
        y = torch.empty(N, g.P, g.Q, K, device="cuda", dtype=torch.bfloat16)
        dy = torch.randn_like(y)
        wt = torch.empty(C, R, S, K, device="cuda", dtype=torch.bfloat16)
        L.dtm_weight_flip_transpose(_lib.ptr(w), _lib.ptr(wt), K, R, S, C, st)
        dx = torch.empty_like(x)
        dw = torch.zeros(K, R, S, C, device="cuda")
        for _ in range(reps):
            assert L.dtm_conv_fwd(_lib.ptr(x), _lib.ptr(w), _lib.ptr(y), None, None, None, None, 0, ctypes.byref(d),
                                  st) == 0
            assert L.dtm_conv_dgrad(_lib.ptr(dy), _lib.ptr(wt), _lib.ptr(dx), ctypes.byref(d), st) == 0
            assert L.dtm_conv_wgrad(_lib.ptr(x), _lib.ptr(dy), _lib.ptr(dw), None, None, ctypes.byref(d),
                                    _lib.num_cus(), st) == 0
        torch.cuda.synchronize()
        print("shape N%d H%d C%d K%d %dx%d done" % (N, H, C, K, R, S), flush=True)


if __name__ == "__main__":
    main()
