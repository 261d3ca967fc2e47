#!/usr/bin/env python3
"""A/B sweep of the conv_nt tile variants (DTM_CONV_TILE ids) on the ResNet-50 shapes, in ONE process
with interleaved rounds (per-shape median over rounds): forward, forward with the BatchNorm-apply
prologue, and dgrad (ACT=1: also the dgrad with the input's BN+ReLU backward epilogue).  Usage: TILES=-1,21,26 python tools/conv_tile_sweep.py"""
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
TILES = [int(t) for t in os.environ.get("TILES", "-1,0,21,24,26,40").split(",")]
ROUNDS = int(os.environ.get("ROUNDS", "3"))
ONLY = os.environ.get("ONLY")


def timed(fn, n=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3  # us


# Inception-v3 (old slim) training shapes at batch 128 (reference inception/slim/inception_model.py:54-332):
# (H, C, K, R, S, stride, padding, count per step)
INCEPTION = [
    (149, 32, 32, 3, 3, 1, "VALID", 1), (147, 32, 64, 3, 3, 1, "SAME", 1), (73, 64, 80, 1, 1, 1, "VALID", 1),
    (73, 80, 192, 3, 3, 1, "VALID", 1),
    (35, 288, 64, 1, 1, 1, "SAME", 9), (35, 288, 48, 1, 1, 1, "SAME", 3), (35, 48, 64, 5, 5, 1, "SAME", 3),
    (35, 64, 96, 3, 3, 1, "SAME", 4), (35, 96, 96, 3, 3, 1, "SAME", 3),
    (35, 288, 384, 3, 3, 2, "VALID", 1), (35, 96, 96, 3, 3, 2, "VALID", 1),
    (17, 768, 192, 1, 1, 1, "SAME", 10), (17, 768, 160, 1, 1, 1, "SAME", 8),
    (17, 160, 160, 1, 7, 1, "SAME", 8), (17, 160, 160, 7, 1, 1, "SAME", 8), (17, 160, 192, 1, 7, 1, "SAME", 4),
    (17, 160, 192, 7, 1, 1, "SAME", 4), (17, 192, 320, 3, 3, 2, "VALID", 1), (17, 192, 192, 3, 3, 2, "VALID", 1),
    (8, 2048, 320, 1, 1, 1, "SAME", 2), (8, 2048, 384, 1, 1, 1, "SAME", 2), (8, 2048, 448, 1, 1, 1, "SAME", 2),
    (8, 2048, 192, 1, 1, 1, "SAME", 2), (8, 384, 384, 1, 3, 1, "SAME", 4), (8, 384, 384, 3, 1, 1, "SAME", 4),
    (8, 448, 384, 3, 3, 1, "SAME", 2),
]


# VGG-16 in the reference's CIFAR geometry (reference vgg/cifar10_vgg_bsp.py:64, vgg/nets/vgg.py:144-222) at batch
# 512; fc6 runs as its live centre tap (1x1), fc7 as a 1x1 conv over a 1x1 map
VGG = [
    (32, 64, 64, 3, 3, 1, "SAME", 1), (16, 64, 128, 3, 3, 1, "SAME", 1), (16, 128, 128, 3, 3, 1, "SAME", 1),
    (8, 128, 256, 3, 3, 1, "SAME", 1), (8, 256, 256, 3, 3, 1, "SAME", 2), (4, 256, 512, 3, 3, 1, "SAME", 1),
    (4, 512, 512, 3, 3, 1, "SAME", 2), (2, 512, 512, 3, 3, 1, "SAME", 3), (1, 512, 4096, 1, 1, 1, "SAME", 1),
    (1, 4096, 4096, 1, 1, 1, "SAME", 1),
]


def main():
    L = _lib.lib()
    st = _lib.stream_ptr()
    print("%-24s %-6s " % ("shape", "pass") + " ".join("%8s" % ("t%d" % t) for t in TILES) + "   best", flush=True)
    tot = {t: 0.0 for t in TILES}
    wtot = {}
    which = os.environ.get("SET", "resnet")
    shapes = ([(H, C, K, R, R, s_, (p_, p_), n) for (H, C, K, R, s_, p_, n) in SHAPES[1:]]
              if which == "resnet" else (INCEPTION if which == "inception" else VGG))
    if which == "custom":  # SHAPES_CUSTOM="H,C,K,R,S,stride,padding,count;..." (e.g. merged sibling-head widths)
        shapes = [tuple(int(v) if v.lstrip("-").isdigit() else v for v in item.split(","))
                  for item in os.environ["SHAPES_CUSTOM"].split(";")]
    for (H, C, K, R, S, stride, pad, cnt) in shapes:
        if ONLY and ONLY not in "%d_%d_%d_%d" % (H, C, K, R):
            continue
        x = torch.randn(B, H, H, C, device="cuda").to(torch.bfloat16)
        w = (torch.randn(K, R, S, C, device="cuda") * 0.05).to(torch.bfloat16)
        g = conv_geom(tuple(x.shape), tuple(w.shape), stride, pad)
        d = g.as_desc(_lib.ConvDesc)
        y = torch.empty(B, g.P, g.Q, K, device="cuda", dtype=torch.bfloat16)
        dy = torch.randn_like(y)
        wt = torch.empty(C, R, S, K, device="cuda", dtype=torch.bfloat16)
        L.dtm_weight_flip_transpose(_lib.ptr(w), _lib.ptr(wt), K, R, S, C, st)
        dx = torch.empty_like(x)
        sc = torch.rand(C, device="cuda") + 0.5
        sh = torch.randn(C, device="cuda") * 0.1
        passes = {
            "fwd": lambda: L.dtm_conv_fwd(_lib.ptr(x), _lib.ptr(w), _lib.ptr(y), None, None, None, None, 0,
                                          ctypes.byref(d), st),
            "fwd+p": lambda: L.dtm_conv_fwd(_lib.ptr(x), _lib.ptr(w), _lib.ptr(y), None, None, _lib.ptr(sc),
                                            _lib.ptr(sh), 0, ctypes.byref(d), st),
            "dgrad": lambda: L.dtm_conv_dgrad(_lib.ptr(dy), _lib.ptr(wt), _lib.ptr(dx), ctypes.byref(d), st),
        }
        if os.environ.get("ACT"):
            # dgrad with the input's BatchNorm+ReLU backward in the epilogue (the bottleneck conv2 / conv3 dgrads)
            ss4 = torch.stack([sc, sh, sh, sc]).contiguous()
            asums = torch.zeros(2, C, device="cuda")
            passes["dgact"] = lambda: L.dtm_conv_dgrad_ex(_lib.ptr(dy), _lib.ptr(wt), _lib.ptr(dx), ctypes.byref(d),
                                                          None, 1, _lib.ptr(x), _lib.ptr(ss4), _lib.ptr(asums), 1, st)
        if stride > 1 and R >= stride and S >= stride:
            # the stride-decomposed dgrad (ConvDesc.dec: one stride-1 conv per output parity class) as training runs it
            wtd = torch.empty(C, R, S, K, device="cuda", dtype=torch.bfloat16)
            L.dtm_weight_flip_transpose_dec(_lib.ptr(w), _lib.ptr(wtd), K, R, S, C, stride, g.pad_h, g.pad_w, st)
            dd = g.as_desc(_lib.ConvDesc)
            dd.dec = 1
            passes["dgdec"] = lambda: L.dtm_conv_dgrad(_lib.ptr(dy), _lib.ptr(wtd), _lib.ptr(dx), ctypes.byref(dd), st)
        if os.environ.get("STATS"):
            stats = torch.zeros(2, K, device="cuda")
            passes["fwd+ps"] = lambda: L.dtm_conv_fwd(_lib.ptr(x), _lib.ptr(w), _lib.ptr(y), _lib.ptr(stats), None,
                                                      _lib.ptr(sc), _lib.ptr(sh), 0, ctypes.byref(d), st)
            passes["fwd+s"] = lambda: L.dtm_conv_fwd(_lib.ptr(x), _lib.ptr(w), _lib.ptr(y), _lib.ptr(stats), None,
                                                     None, None, 0, ctypes.byref(d), st)
        if os.environ.get("WGRAD"):
            dw = torch.zeros(K, R, S, C, device="cuda")
            ss4 = torch.stack([sc, sh, sh, sc]).contiguous()
            mask = torch.empty(x.numel() // 8, device="cuda", dtype=torch.uint8)
            xa = torch.empty_like(x)
            ext = {
                "wgrad": lambda: L.dtm_conv_wgrad(_lib.ptr(x), _lib.ptr(dy), _lib.ptr(dw), None, None, ctypes.byref(d),
                                                  _lib.num_cus(), st),
                "wgrad+p": lambda: L.dtm_conv_wgrad(_lib.ptr(x), _lib.ptr(dy), _lib.ptr(dw), _lib.ptr(sc), _lib.ptr(sh),
                                                    ctypes.byref(d), _lib.num_cus(), st),
                "apply": lambda: L.dtm_bn_apply2(_lib.ptr(x), _lib.ptr(ss4), None, None, _lib.ptr(xa), _lib.ptr(mask),
                                                 x.numel() // C, C, 0, 1, st),
            }
            for pname, fn in ext.items():
                v = statistics.median([timed(fn) for _ in range(ROUNDS)])
                print("H%-3d C%-4d K%-4d R%d s%d x%d %-7s %8.1f" % (H, C, K, R, stride, cnt, pname, v), flush=True)
        if os.environ.get("WTILES"):
            wts = [tuple(int(u) for u in t.split(":")) for t in os.environ["WTILES"].split(",")]
            dw = torch.zeros(K, R, S, C, device="cuda")
            pro = (_lib.ptr(sc), _lib.ptr(sh)) if os.environ.get("WPRO") else (None, None)  # BN-apply prologue on x
            fn = lambda: L.dtm_conv_wgrad(_lib.ptr(x), _lib.ptr(dy), _lib.ptr(dw), pro[0], pro[1],  # noqa
                                          ctypes.byref(d), _lib.num_cus(), st)
            res = {t: [] for t in wts}
            for _ in range(ROUNDS):
                for t in wts:
                    L.dtm_conv_set_wgrad_tile(t[0], t[1] if len(t) > 1 else 0)
                    res[t].append(timed(fn))
            L.dtm_conv_set_wgrad_tile(-1, 4)
            med = {t: statistics.median(v) for t, v in res.items()}
            for t in wts:
                wtot[t] = wtot.get(t, 0.0) + med[t] * cnt
            print("H%-3d C%-4d K%-4d R%d s%d x%d %-6s " % (H, C, K, R, stride, cnt, "wgrad") +
                  " ".join("%s=%.1f" % (":".join(map(str, t)), med[t]) for t in wts), flush=True)
            if os.environ.get("WONLY"):
                continue
        for pname, fn in passes.items():
            res = {t: [] for t in TILES}
            for _ in range(ROUNDS):
                for t in TILES:
                    L.dtm_conv_set_tile(t)
                    res[t].append(timed(fn))
            L.dtm_conv_set_tile(-1)
            med = {t: statistics.median(v) for t, v in res.items()}
            for t in TILES:
                tot[t] += med[t] * cnt
            best = min(med, key=med.get)
            print("H%-3d C%-4d K%-4d R%dx%d s%d x%d %-6s " % (H, C, K, R, S, stride, cnt, pname) +
                  " ".join("%8.1f" % med[t] for t in TILES) + "   t%d" % best, flush=True)
    print("weighted total (us): " + " ".join("t%d=%.0f" % (t, v) for t, v in tot.items()), flush=True)
    if wtot:
        print("wgrad weighted total (us): " + " ".join("%s=%.0f" % (":".join(map(str, t)), v) for t, v in wtot.items()))


if __name__ == "__main__":
    main()
