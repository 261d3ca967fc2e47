#!/usr/bin/env python3
"""Library-GEMM reference for the ResNet-50 implicit-GEMM conv shapes: torch.matmul (hipBLASLt) on the equivalent
bf16 GEMM (M = N*P*Q pixels, N = output channels, K = R*S*C) next to our conv kernel on the conv itself, same
process, random operands, interleaved rounds.  What a tuned library tile reaches on these shapes is the ceiling the
hand-written tiles are measured against (cdna_hip_programming.md rule 10).  Usage: python tools/gemm_ref_bench.py"""
import ctypes
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_tensorflow_models_amd.ops import _lib  # noqa: E402
from distributed_tensorflow_models_amd.ops.geometry import conv_geom  # noqa: E402

# (H, C, K, R) at batch 256, stride 1
SHAPES = [(14, 256, 256, 3), (7, 512, 512, 3), (28, 128, 128, 3), (14, 1024, 256, 1), (7, 1024, 2048, 1),
          (28, 128, 512, 1), (56, 64, 256, 1), (14, 256, 1024, 1), (7, 2048, 512, 1)]
B = int(os.environ.get("B", "256"))
TILES = [int(t) for t in os.environ.get("TILES", "-1").split(",")]


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
    print("%-20s %10s %8s " % ("shape", "gemm_us", "gemm_TF") + " ".join("%12s" % ("t%d us/TF" % t) for t in TILES))
    for (H, C, K, R) in SHAPES:
        M, Kg = B * H * H, R * R * C
        a = torch.randn(M, Kg, device="cuda").to(torch.bfloat16)
        bm = torch.randn(Kg, K, device="cuda").to(torch.bfloat16)
        out = torch.empty(M, K, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(B, H, H, C, device="cuda").to(torch.bfloat16)
        w = (torch.randn(K, R, R, C, device="cuda") * 0.05).to(torch.bfloat16)
        g = conv_geom(tuple(x.shape), tuple(w.shape), 1, "SAME")
        d = g.as_desc(_lib.ConvDesc)
        y = torch.empty(B, g.P, g.Q, K, device="cuda", dtype=torch.bfloat16)
        fl = 2.0 * M * K * Kg
        res = {"gemm": []}
        for t in TILES:
            res[t] = []
        for _ in range(int(os.environ.get("ROUNDS", "3"))):
            res["gemm"].append(timed(lambda: torch.matmul(a, bm, out=out)))
            for t in TILES:
                L.dtm_conv_set_tile(t)
                res[t].append(timed(lambda: L.dtm_conv_fwd(_lib.ptr(x), _lib.ptr(w), _lib.ptr(y), None, None, None,
                                                           None, 0, ctypes.byref(d), st)))
        L.dtm_conv_set_tile(-1)
        med = {k: statistics.median(v) for k, v in res.items()}
        print("H%-2d C%-4d K%-4d R%d    %10.1f %8.0f " % (H, C, K, R, med["gemm"], fl / med["gemm"] / 1e6) +
              " ".join("%6.1f/%5.0f" % (med[t], fl / med[t] / 1e6) for t in TILES), flush=True)


if __name__ == "__main__":
    main()
