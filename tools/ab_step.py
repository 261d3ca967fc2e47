#!/usr/bin/env python3
"""Same-process A/B of whole ResNet-50 training steps under kernel-policy variants (interleaved rounds,
median ms/step per variant; one device, one process: MI355X_MICROARCH 'DVFS give-back' / rule 24).

VARIANTS="base=;noW=wtile:-3;noT=tile:-3;fused=prologue:fused" python tools/ab_step.py
keys: tile (conv_nt tile id), w8 (0/1: the 8-wave 256x256 conv tile in the shape policy), pp (0/1: its ping-pong
form conv_nt_pp_kernel in place of conv_nt_w8_kernel), ct32 (0/1: 32-channel output tiles of the direct 3x3 kernel
for K = 64), wdir (0/1: the direct 3x3 weight gradient for 32 input channels), sbna (0/1: the stem's BN-fused wgrad on the pipelined
64x256 tile), aocc (0-3: occupancy variants of the register-staged dgrads with post-ops), nocc (the same for
their launches without side inputs), kwide (0/1: 64-channel
tiles for K % 128 <= 64), few (0/1: streaming few-row slab reduction), sact (0/1: streaming 1x1 kernel for act
dgrads), k32 (0/1: 256x32 tile for <=32-channel spatial convs), cpt (16-B chunks per thread of the BN-stream grids),
pol2 (0/1: v2 conv tile-policy rules), sstr (0/1/2: the stem forward as a persistent stream, 3- / 2-slot ring), wgs
(0/1: conv+BN weight gradients on a side stream), scu (percent of the CUs the side-stream wgrads size their split-K
grid for), wcu / swc (the same for the main-stream / stem wgrads), dir3 (0/1: direct 3x3 kernel for C in {32, 64}),
dgrp (0/1: strided-dgrad parity classes as one grouped launch), atile (tile id of the dgrads with a fused
activation-backward epilogue, -1 = policy), rsv (CUs reserved from the compute grids' sizing), lpt (0/1: grouped
parity classes in descending tap count), dtile (0/1: grouped strided-dgrad tile chosen for the whole grouped grid),
stile (0/1: merged-head convs on the pipelined 128x128 tile), fdir (0/1: one-block BN finalize when one row
chunk covers every statistics row), hog (blocks:ms - a CU-occupying copy kernel on another
stream from every backward start, standing in for RCCL channels), wtile[:occ] (wgrad tile id / blocks-per-CU target),
prologue (auto | fused | mat | apply: ops/fused.py PROLOGUE_MODE), red (target_blocks:max_chunks[:direct_max] of the
partial-sum reductions), off (name+name: fused-path features of ops/features.py switched off, e.g.
off:sibling_fwd+act_handoff)."""
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_tensorflow_models_amd.engine import TrainStep  # noqa: E402
from distributed_tensorflow_models_amd.models import nets_factory  # noqa: E402
from distributed_tensorflow_models_amd.ops import _lib, features, fused  # noqa: E402


HOG = [None]  # "blocks:ms": CU-contention stand-in for RCCL channels launched at every backward start


def _hog():
    if not HOG[0]:
        return
    n, ms = HOG[0].split(":")
    st = _HOG_STREAM[0]
    if st is None:
        st = _HOG_STREAM[0] = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    rc = _lib.lib().dtm_cu_hog(int(n), float(ms), _lib.ctypes.c_void_p(st.cuda_stream))
    assert rc == 0, rc


_HOG_STREAM = [None]
WGS_DEFAULT = ["1"]  # (the model preset's choice, set in main)


def apply(cfg):
    L = _lib.lib()
    L.dtm_conv_set_tile(int(cfg.get("tile", -1)))
    wt = cfg.get("wtile", "-1").split(":")
    L.dtm_conv_set_wgrad_tile(int(wt[0]), int(wt[1]) if len(wt) > 1 else 0)
    red = cfg.get("red", "0:64:0").split(":")
    L.dtm_set_reduce_policy(int(red[0]), int(red[1]), int(red[2]) if len(red) > 2 else 0)
    L.dtm_set_ntld_policy(int(cfg.get("ntld", "3")))
    L.dtm_set_deterministic(int(cfg.get("det", "0")))
    L.dtm_conv_set_k64_tile(int(cfg.get("k64", "3")))
    L.dtm_conv_set_w8(int(cfg.get("w8", "1")))
    L.dtm_conv_set_pp(int(cfg.get("pp", "0")))
    L.dtm_conv_set_direct_ct32(int(cfg.get("ct32", "1")))
    L.dtm_conv_set_wgrad_direct(int(cfg.get("wdir", "1")), 0)
    L.dtm_conv_set_stem_bna(int(cfg.get("sbna", "1")))
    L.dtm_conv_set_act_occ(int(cfg.get("aocc", "2")))
    L.dtm_conv_set_nt_occ(int(cfg.get("nocc", "2")))
    L.dtm_conv_set_kwide(int(cfg.get("kwide", "1")))
    L.dtm_set_reduce_few(int(cfg.get("few", "1")))
    L.dtm_conv_set_stream_act(int(cfg.get("sact", "0")))
    L.dtm_conv_set_act_tile(int(cfg.get("atile", "-1")))
    L.dtm_conv_set_policy2(int(cfg.get("pol2", "1")))
    L.dtm_set_grid_cpt(int(cfg.get("cpt", "8")))
    L.dtm_conv_set_k32(int(cfg.get("k32", "1")))
    L.dtm_conv_set_stem_stream(int(cfg.get("sstr", "1")))
    _lib.set_side_enabled(cfg.get("wgs", WGS_DEFAULT[0]) == "1")
    _lib.set_side_cu_fraction(float(cfg.get("scu", "75")) / 100.0)
    _lib.set_wgrad_cu_percent("main", cfg.get("wcu", "100"))
    _lib.set_wgrad_cu_percent("stem", cfg.get("swc", "100"))
    L.dtm_conv_set_direct3(int(cfg.get("dir3", "1")))
    L.dtm_conv_set_dec_group(int(cfg.get("dgrp", "1")))
    _lib.set_reserved_cus(int(cfg.get("rsv", "0")))
    L.dtm_conv_set_dec_lpt(int(cfg.get("lpt", "1")))
    L.dtm_conv_set_dec_tile(int(cfg.get("dtile", "1")))
    L.dtm_conv_set_split_tile(int(cfg.get("stile", "1")))
    L.dtm_set_fin_direct(int(cfg.get("fdir", "1")))
    HOG[0] = cfg.get("hog")
    sc = cfg.get("sc", "5:4096").split(":")
    L.dtm_set_sc_policy(int(sc[0]), int(sc[1]))
    fused.PROLOGUE_MODE = None if cfg.get("prologue", "auto") == "auto" else cfg["prologue"]
    # fused-path features (ops/features.py) switched off by this variant: off:<name>+<name>
    os.environ["DTM_DISABLE"] = ",".join(n for n in cfg.get("off", "").split("+") if n)
    features.check_env()


def main():
    variants = []
    for item in os.environ.get("VARIANTS", "base=").split(";"):
        name, _, spec = item.partition("=")
        cfg = dict(kv.split(":", 1) for kv in spec.split(",") if kv)
        variants.append((name, cfg))
    B = int(os.environ.get("B", "0"))
    steps, rounds = int(os.environ.get("STEPS", "6")), int(os.environ.get("ROUNDS", "4"))
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = os.environ.get("MODEL", "resnet_v1_50")
    from bench import PRESETS
    S, ncls, B0, opt, extra = PRESETS[model]
    if "wgrad_stream" in extra:
        WGS_DEFAULT[0] = "1" if extra["wgrad_stream"] else "0"
    kw = {"fc_conv_padding": "SAME"} if model == "vgg_16" else {}  # (bench.py's CIFAR geometry)
    net = nets_factory.build(model, num_classes=ncls, **kw).to(dev)
    B = B or B0
    # (eager steps only: captured hipGraphs of several variants in one process hold raw pointers into scratch
    # that a later variant's eager warm-up may reallocate - two such runs faulted, profiles/ab/README.md)
    step = TrainStep(net, optimizer=opt, lr=0.01, momentum=0.9, **extra)
    step.on_backward = _hog
    x = torch.randn(B, S, S, 1 if model == "lenet" else 3, device=dev).to(torch.bfloat16)
    y = torch.randint(0, ncls, (B,), device=dev)
    res = {n: [] for n, _ in variants}
    for n, cfg in variants:  # warm every variant (workspace growth, first-touch)
        apply(cfg)
        for _ in range(2):
            step(x, y)
    torch.cuda.synchronize()
    for r in range(rounds):
        for n, cfg in variants:
            apply(cfg)
            step(x, y)
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(steps):
                step(x, y)
            torch.cuda.synchronize()
            res[n].append((time.perf_counter() - t) / steps * 1e3)
        print("round %d: " % r + " ".join("%s=%.3f" % (n, res[n][-1]) for n, _ in variants), flush=True)
    base = statistics.median(res[variants[0][0]])
    for n, _ in variants:
        m = statistics.median(res[n])
        print("%-10s median %.3f ms/step  min %.3f  (%+.2f %% vs %s)  %.0f img/s" % (
            n, m, min(res[n]), (m / base - 1) * 100, variants[0][0], B / m * 1e3), flush=True)
    apply({})


if __name__ == "__main__":
    main()
