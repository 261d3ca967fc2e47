#!/usr/bin/env python3
"""Which Python call sites still launch PyTorch (aten) device kernels inside one training step.

Runs a bench preset for a few eager steps, then profiles one step with torch.profiler (CPU op
events + Python stacks) and prints, per aten op that launched device work, the innermost frame of
this package that called it, with the call count per step.  Usage:
    python tools/aten_sites.py [--model inception_v3_slim_old] [--batch 128]
"""
import argparse
import os
import sys
from collections import Counter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="inception_v3_slim_old")
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--dispatch", action="store_true",
                    help="attribute ops with a TorchDispatchMode + Python traceback (works in custom backward)")
    args = ap.parse_args()
    import torch
    from torch.profiler import ProfilerActivity, profile

    import bench
    from distributed_tensorflow_models_amd.engine import TrainStep
    from distributed_tensorflow_models_amd.models import nets_factory

    S, ncls, B0, opt, extra = bench.PRESETS[args.model]
    B = args.batch or B0
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    kw = {"fc_conv_padding": "SAME"} if args.model == "vgg_16" else {}
    net = nets_factory.build(args.model, num_classes=ncls, **kw).to(dev)
    step = TrainStep(net, optimizer=opt, lr=0.01, momentum=0.9, **extra)
    cin = 1 if args.model == "lenet" else 3
    x = torch.randn(B, S, S, cin, device=dev).to(torch.bfloat16)
    y = torch.randint(0, ncls, (B,), device=dev)
    for _ in range(3):
        step(x, y)
    torch.cuda.synchronize()
    if args.dispatch:
        return dispatch_sites(step, x, y)
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        step(x, y)
        torch.cuda.synchronize()
    sites = Counter()
    dev_us = Counter()
    pkg = "distributed_tensorflow_models_amd"
    for ev in prof.events():
        if not ev.name.startswith("aten::") or ev.device_type.name != "CPU":
            continue
        if ev.cpu_parent is not None and ev.cpu_parent.name.startswith("aten::"):
            continue  # count the outermost aten op only
        kern = sum(k.duration for k in ev.kernels) if ev.kernels else 0
        if kern == 0 and ev.device_time_total == 0:
            continue
        frame = next((f for f in (ev.stack or []) if pkg in f or "bench.py" in f), None)
        par = ev.cpu_parent
        while frame is None and par is not None:  # python_function events of the tracer
            if pkg in par.name and ".py(" in par.name:
                frame = par.name
            par = par.cpu_parent
        frame = frame or "?"
        key = (ev.name, frame.split(pkg + "/")[-1])
        sites[key] += 1
        dev_us[key] += ev.device_time_total
    print("%-28s %5s %9s  %s" % ("aten op", "calls", "dev us", "call site"))
    for key, n in sorted(sites.items(), key=lambda kv: -dev_us[kv[0]]):
        print("%-28s %5d %9.1f  %s" % (key[0], n, dev_us[key], key[1]))
    print("total aten device us/step: %.1f" % sum(dev_us.values()))


def dispatch_sites(step, x, y):
    """Every aten op of one step whose outputs live on the GPU, keyed by the innermost package frame."""
    import traceback

    import torch
    from torch.utils._python_dispatch import TorchDispatchMode
    skip = ("aten::empty", "aten::view", "aten::as_strided", "aten::detach", "aten::alias",
            "aten::_unsafe_view", "aten::t", "aten::reshape", "aten::slice", "aten::select", "aten::expand",
            "aten::permute", "aten::unsqueeze", "aten::squeeze", "aten::empty_strided", "aten::lift_fresh",
            "aten::set_", "aten::resize_", "aten::split", "aten::is_same_size")
    pkg = "distributed_tensorflow_models_amd"
    sites = Counter()

    class Mode(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            out = func(*args, **(kwargs or {}))
            name = "aten::" + func.__name__.split(".")[0]
            if name not in skip:
                outs = out if isinstance(out, (tuple, list)) else [out]
                if any(isinstance(o, torch.Tensor) and o.is_cuda for o in outs):
                    fr = [f for f in traceback.extract_stack()[:-1] if pkg in f.filename or "bench" in f.filename]
                    site = ("%s:%d %s" % (fr[-1].filename.split(pkg + "/")[-1], fr[-1].lineno, fr[-1].name)
                            if fr else "(autograd engine)")
                    sites[(func.__name__, site)] += 1
            return out

    with Mode():
        step(x, y)
    torch.cuda.synchronize()
    print("%-34s %5s  %s" % ("aten op", "calls", "innermost package frame"))
    for (op, site), n in sorted(sites.items(), key=lambda kv: -kv[1]):
        print("%-34s %5d  %s" % (op, n, site))


if __name__ == "__main__":
    main()
