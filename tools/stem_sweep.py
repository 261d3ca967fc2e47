#!/usr/bin/env python3
"""Tile sweep of the ResNet-50 stem (7x7/2 conv, 3 -> 64 channels, 224x224, packed-row view of
_StemConvBNFn) - forward with BN statistics and the weight gradient - in one process, interleaved
rounds, median per variant.  TILES / WTILES env: comma lists (wgrad entries id[:occ]).  INC=1: Inception-v3's
stem instead (3x3/2 VALID, 3 -> 32 channels, 299x299, batch 128)."""
import ctypes
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_tensorflow_models_amd.ops import _lib  # noqa: E402

INC = os.environ.get("INC") == "1"
B = int(os.environ.get("B", "128" if INC else "256"))
TILES = [int(t) for t in os.environ.get("TILES", "-1,1,3,12,23,24,25,26").split(",")]
WTILES = os.environ.get("WTILES", "-1,1,2,13:2,14:1,15:2,15:4").split(",")
ROUNDS = int(os.environ.get("ROUNDS", "3"))


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
    # (the packed geometry of ops/fused.py _StemConvBNFn)
    K, R, Hp, Wp, P = (32, 3, 299, 304, 149) if INC else (64, 7, 230, 230, 112)
    Q = P
    xp = torch.randn(B, Hp, Wp, 4, device="cuda").to(torch.bfloat16)
    wv = (torch.randn(K, R, 8, 4, device="cuda") * 0.05).to(torch.bfloat16)
    d = _lib.ConvDesc(B, Hp, Wp, 32, K, R, 1, P, Q, 2, 0, 0, 8)
    y = torch.empty(B, P, Q, K, device="cuda", dtype=torch.bfloat16)
    stats = torch.zeros(2, K, device="cuda")
    dy = torch.randn_like(y)
    dw = torch.zeros(K, R, 8, 4, device="cuda")
    res = {("fwd+s", t): [] for t in TILES}
    res.update({("wgrad", w): [] for w in WTILES})
    res.update({("wg+bn", w): [] for w in WTILES})
    # the training form: the BN backward of dy fused into the wgrad's operand staging (dtm_conv_wgrad_bnbwd)
    dss = torch.randn(4, K, device="cuda") * 1e-3
    ss = torch.cat([torch.rand(1, K, device="cuda") + 0.5, torch.randn(3, K, device="cuda")]).contiguous()
    gamma = torch.rand(K, device="cuda") + 0.5
    dg, db = torch.zeros(K, device="cuda"), torch.zeros(K, device="cuda")
    for _ in range(ROUNDS):
        for t in TILES:
            L.dtm_conv_set_tile(t)
            res[("fwd+s", t)].append(timed(lambda: L.dtm_conv_fwd(_lib.ptr(xp), _lib.ptr(wv), _lib.ptr(y),
                                                                   _lib.ptr(stats), None, None, None, 0,
                                                                   ctypes.byref(d), st)))
        L.dtm_conv_set_tile(-1)
        for w in WTILES:
            i, _, o = w.partition(":")
            L.dtm_conv_set_wgrad_tile(int(i), int(o or 0))
            res[("wgrad", w)].append(timed(lambda: L.dtm_conv_wgrad(_lib.ptr(xp), _lib.ptr(dy), _lib.ptr(dw), None,
                                                                     None, ctypes.byref(d), _lib.num_cus(), st)))
            res[("wg+bn", w)].append(timed(lambda: L.dtm_conv_wgrad_bnbwd(
                _lib.ptr(xp), _lib.ptr(dy), _lib.ptr(y), _lib.ptr(dss), _lib.ptr(ss), _lib.ptr(gamma), float(B * P * Q),
                _lib.ptr(dg), _lib.ptr(db), _lib.ptr(dw), ctypes.byref(d), _lib.num_cus(), st)))
        L.dtm_conv_set_wgrad_tile(-1, 4)
    for (p, t), v in res.items():
        print("stem %-6s %-6s %8.1f us" % (p, t, statistics.median(v)), flush=True)


if __name__ == "__main__":
    main()
