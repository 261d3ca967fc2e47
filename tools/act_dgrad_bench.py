#!/usr/bin/env python3
"""Per-tile timing of the block-output dgrads of ResNet-50 (dtm_conv_dgrad_bnout: dgrad of a unit's conv1 + the
residual gradient add + the block-output ReLU mask + the BN-backward partial sums), the step's
'add=1 act=1 mask=1' conv launches, with the HBM floor of each (bytes moved / 5.5 TB/s).  Interleaved rounds in one
process.  Usage: TILES=-1,4,40,21 python tools/act_dgrad_bench.py"""
import ctypes
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_tensorflow_models_amd.ops import _lib  # noqa: E402
from distributed_tensorflow_models_amd.ops.geometry import conv_geom  # noqa: E402

B = int(os.environ.get("B", "256"))
TILES = [int(t) for t in os.environ.get("TILES", "-1,4,40,21,24").split(",")]
# optional knob sweep: KNOB=<dtm_* setter> VALUES=a,b,...: every tile is timed under every value
KNOB = os.environ.get("KNOB")
VALUES = [int(v) for v in os.environ.get("VALUES", "0").split(",")]
# forward conv1 shapes (H, C = block width, K = bottleneck width): its dgrad writes the C-channel block gradient
SHAPES = [(56, 256, 64), (28, 512, 128), (14, 1024, 256), (7, 2048, 512)]


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
    knob = getattr(L, KNOB) if KNOB else (lambda v: None)
    cols = [(t, v) for t in TILES for v in VALUES]
    print("%-18s %8s " % ("shape", "floor") + " ".join("%8s" % ("t%dv%d" % c) for c in cols))
    for (H, C, K) in SHAPES:
        x = torch.randn(B, H, H, C, device="cuda").to(torch.bfloat16)
        w = (torch.randn(K, 1, 1, C, device="cuda") * 0.05).to(torch.bfloat16)
        g = conv_geom(tuple(x.shape), tuple(w.shape), 1, "SAME")
        d = g.as_desc(_lib.ConvDesc)
        dy = torch.randn(B, H, H, K, device="cuda").to(torch.bfloat16)
        wt = torch.empty(C, 1, 1, K, device="cuda", dtype=torch.bfloat16)
        L.dtm_weight_flip_transpose(_lib.ptr(w), _lib.ptr(wt), K, 1, 1, C, st)
        add = torch.randn_like(x)
        mask = torch.randint(0, 256, (x.numel() // 8,), device="cuda", dtype=torch.uint8)
        sums = torch.zeros(2, C, device="cuda")
        dx = torch.empty_like(x)
        nbytes = dy.numel() * 2 + 3 * x.numel() * 2 + mask.numel()
        fn = lambda: L.dtm_conv_dgrad_bnout(_lib.ptr(dy), _lib.ptr(wt), _lib.ptr(dx), ctypes.byref(d),  # noqa: E731
                                            _lib.ptr(add), 1, _lib.ptr(mask), _lib.ptr(x), None, _lib.ptr(sums), st)
        res = {c: [] for c in cols}
        for _ in range(int(os.environ.get("ROUNDS", "3"))):
            for c in cols:
                L.dtm_conv_set_tile(c[0])
                knob(c[1])
                res[c].append(timed(fn))
        L.dtm_conv_set_tile(-1)
        knob(VALUES[0])
        print("H%-2d C%-4d K%-4d    %8.1f " % (H, C, K, nbytes / 5.5e12 * 1e6) +
              " ".join("%8.1f" % statistics.median(res[c]) for c in cols), flush=True)


if __name__ == "__main__":
    main()
