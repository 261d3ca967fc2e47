#!/usr/bin/env python3
"""Same-process A/B of a kernel-policy knob on single conv launches (interleaved rounds, median per variant).

KNOB=dtm_conv_set_w8_stag VALUES=0,1 TILE=40 SET=resnet PASSES=fwd,dgrad python tools/knob_ab.py
The conv tile is forced to TILE (-1 = policy) for every launch; the knob function is called with each value before
its timed block.  Shapes: tools/conv_microbench.py SHAPES (ResNet-50, batch 256) filtered by ONLY (substring of
'H_C_K_R')."""
import ctypes
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_tensorflow_models_amd.ops import _lib  # noqa: E402
from distributed_tensorflow_models_amd.ops.geometry import conv_geom  # noqa: E402
from tools.conv_microbench import SHAPES  # noqa: E402

B = int(os.environ.get("B", "256"))


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
    knob = getattr(L, os.environ["KNOB"])
    values = [int(v) for v in os.environ.get("VALUES", "0,1").split(",")]
    tile = int(os.environ.get("TILE", "-1"))
    passes = os.environ.get("PASSES", "fwd,dgrad").split(",")
    only = os.environ.get("ONLY")
    rounds = int(os.environ.get("ROUNDS", "5"))
    tot = {v: 0.0 for v in values}
    print("%-26s %-6s " % ("shape", "pass") + " ".join("%9s" % ("v=%d" % v) for v in values))
    L.dtm_conv_set_tile(tile)
    for (H, C, K, R, s_, p_, cnt) in SHAPES[1:]:
        if only and not any(o in "%d_%d_%d_%d" % (H, C, K, R) for o in only.split(",")):
            continue
        x = torch.randn(B, H, H, C, device="cuda").to(torch.bfloat16)
        w = (torch.randn(K, R, R, C, device="cuda") * 0.05).to(torch.bfloat16)
        g = conv_geom(tuple(x.shape), tuple(w.shape), s_, (p_, p_))
        d = g.as_desc(_lib.ConvDesc)
        y = torch.empty(B, g.P, g.Q, K, device="cuda", dtype=torch.bfloat16)
        dy = torch.randn_like(y)
        wt = torch.empty(C, R, R, K, device="cuda", dtype=torch.bfloat16)
        L.dtm_weight_flip_transpose(_lib.ptr(w), _lib.ptr(wt), K, R, R, C, st)
        dx = torch.empty_like(x)
        dw = torch.zeros(K, R, R, C, device="cuda")
        stats = torch.zeros(2, K, device="cuda")
        fns = {
            "fwd": lambda: L.dtm_conv_fwd(_lib.ptr(x), _lib.ptr(w), _lib.ptr(y), _lib.ptr(stats), None, None, None, 0,
                                          ctypes.byref(d), st),
            "dgrad": lambda: L.dtm_conv_dgrad(_lib.ptr(dy), _lib.ptr(wt), _lib.ptr(dx), ctypes.byref(d), st),
            "wgrad": lambda: L.dtm_conv_wgrad(_lib.ptr(x), _lib.ptr(dy), _lib.ptr(dw), None, None, ctypes.byref(d),
                                              _lib.num_cus(), st),
        }
        for pn in passes:
            if s_ > 1 and pn == "dgrad":
                continue
            res = {v: [] for v in values}
            for _ in range(rounds):
                for v in values:
                    knob(v)
                    res[v].append(timed(fns[pn]))
            med = {v: statistics.median(r) for v, r in res.items()}
            for v in values:
                tot[v] += med[v] * cnt
            print("H%-3d C%-4d K%-4d R%d s%d x%d %-6s " % (H, C, K, R, s_, cnt, pn) +
                  " ".join("%9.1f" % med[v] for v in values), flush=True)
    L.dtm_conv_set_tile(-1)
    print("weighted total (us): " + " ".join("v=%d %.0f" % (v, t) for v, t in tot.items()))


if __name__ == "__main__":
    main()
