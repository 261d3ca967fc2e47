#!/usr/bin/env python3
"""Gradient agreement of the block-output BN backward fused into the dgrad epilogue vs the separate
bn_apply_bwd pass, next to the run-to-run noise of the unfused path (fp32 atomics in the BN sums).
Usage: python tools/diag_bnout.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from distributed_tensorflow_models_amd.models import nets_factory
    from distributed_tensorflow_models_amd.ops import fused
    from distributed_tensorflow_models_amd.ops import nn as F
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    net = nets_factory.build("resnet_v1_50", num_classes=10).to(dev)
    x = torch.randn(int(os.environ.get("B", "4")), 64, 64, 3, device=dev).to(torch.bfloat16)
    y = torch.randint(0, 10, (x.shape[0],), device=dev)
    runs = {}
    for tag, fuse in (("u1", "0"), ("u2", "0"), ("f", "1")):
        os.environ["DTM_DISABLE"] = "" if fuse == "1" else "bnout_fuse"
        for p in net.parameters():
            p.grad = None
        n0 = fused.BNOUT_FUSED[0]
        F.softmax_cross_entropy(net(x, training=True), y).mean().backward()
        torch.cuda.synchronize()
        runs[tag] = {n: p.grad.detach().float().clone() for n, p in net.named_parameters() if p.grad is not None}
        print(tag, "fused units:", fused.BNOUT_FUSED[0] - n0)

    # CPU fp32 reference of the same weights / batch (ops/reference.py path)
    import copy
    cpu = copy.deepcopy(net).cpu()
    for p in cpu.parameters():
        p.grad = None
        if hasattr(p, "bf16"):
            del p.bf16
    F.softmax_cross_entropy(cpu(x.cpu().float(), training=True), y.cpu()).mean().backward()
    runs["cpu"] = {n: p.grad.detach().float().clone().to(dev) for n, p in cpu.named_parameters() if p.grad is not None}

    def rel(a, b):
        return ((a - b).norm() / (b.norm() + 1e-12)).item()
    rows = sorted(((rel(runs["f"][k], runs["u1"][k]), rel(runs["u2"][k], runs["u1"][k]), k) for k in runs["u1"]),
                  reverse=True)
    print("%-60s %10s %10s" % ("param", "fused-vs-u", "u-vs-u"))
    for r in rows[:12]:
        print("%-60s %10.2e %10.2e" % (r[2], r[0], r[1]))
    import re
    per = {}
    for e, _n, k in rows:
        m = re.match(r"units\.(\d+)\.", k)
        u = int(m.group(1)) if m else -1
        per[u] = max(per.get(u, 0.0), e)
    print("max fused-vs-unfused rel error per unit (-1 = stem / logits):")
    print(" ".join("%d:%.1e" % (u, per[u]) for u in sorted(per)))
    import statistics
    eu = [rel(runs["u1"][k], runs["cpu"][k]) for k in runs["cpu"]]
    ef = [rel(runs["f"][k], runs["cpu"][k]) for k in runs["cpu"]]
    print("vs CPU fp32: unfused median %.3e max %.3e | fused median %.3e max %.3e" % (
        statistics.median(eu), max(eu), statistics.median(ef), max(ef)))
    worse = sum(1 for a, b in zip(ef, eu) if a > b)
    print("params where fused is further from fp32 than unfused: %d of %d" % (worse, len(ef)))


if __name__ == "__main__":
    main()
