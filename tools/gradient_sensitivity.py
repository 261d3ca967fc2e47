#!/usr/bin/env python3
"""How chaotic is a random-init network's gradient?  CPU fp32 (ops/reference.py): the step-1 gradient of every
parameter at the unperturbed batch vs the same batch with a relative input perturbation eps (x * (1 + eps * n),
n ~ N(0, 1)); per-tensor relative difference |g_eps - g| / |g| (median / p90 / max over tensors, and a few named
tensors from stem to logits).  A well-conditioned network moves its gradient by O(eps); the random-init
old-slim Inception-v3 (BatchNorm after every conv, no residual path) moves it by ~4e4 x eps at the stem and
~1e2 x eps at the logits, at any batch size - the BatchNorm gradient explosion at initialisation - so bf16 rounding
(eps ~ 4e-3) alone decorrelates its deep-layer gradients from fp32 (tests/test_trajectory_inception_gpu.py).

Usage: python tools/gradient_sensitivity.py MODEL IMAGE BATCH EPS [EPS ...]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def grads(model, x, y, eps, ncls):
    from distributed_tensorflow_models_amd.engine import TrainStep
    from distributed_tensorflow_models_amd.models import nets_factory
    torch.manual_seed(0)
    kw = dict(dropout_keep_prob=1.0) if "inception" in model else {}
    net = nets_factory.build(model, num_classes=ncls, **kw)
    inc = "inception" in model
    step = TrainStep(net, optimizer="sgd", lr=0.0, label_smoothing=0.1 if inc else 0.0, aux_weight=0.4,
                     wgrad_stream=False)
    g = torch.Generator().manual_seed(5)
    xx = x * (1 + eps * torch.randn(x.shape, generator=g)) if eps else x
    loss, _ = step._forward_backward(xx, y)
    return float(loss), {k: p.main_grad.clone() for k, p in net.named_parameters()}


def main():
    model, S, B = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    epss = [float(e) for e in sys.argv[4:]] or [1e-6, 1e-4]
    torch.set_num_threads(os.cpu_count() or 8)
    ncls = 1001 if "inception" in model else 1000
    g = torch.Generator().manual_seed(3)
    x = torch.randn(B, S, S, 3, generator=g).to(torch.bfloat16).float()
    y = torch.randint(1, 11, (B,), generator=g)
    l0, g0 = grads(model, x, y, 0.0, ncls)
    names = [k for k in g0 if g0[k].norm() > 0]
    print("%s %dx%d batch %d: loss %.6f, %d parameter tensors with a gradient" % (model, S, S, B, l0, len(names)))
    for eps in epss:
        l1, g1 = grads(model, x, y, eps, ncls)
        r = sorted((float((g1[k] - g0[k]).norm() / g0[k].norm()), k) for k in names)
        print("eps %.0e: loss %.6f; per-tensor gradient rel diff median %.3g (%.3g x eps) p90 %.3g max %.3g (%s)" % (
            eps, l1, r[len(r) // 2][0], r[len(r) // 2][0] / eps, r[int(0.9 * (len(r) - 1))][0], r[-1][0], r[-1][1]))
        order = list(g0)
        for k in (order[0], order[len(order) // 4], order[len(order) // 2], order[3 * len(order) // 4], order[-1]):
            if k in names:
                print("    %-60s %.3g" % (k, float((g1[k] - g0[k]).norm() / g0[k].norm())))
        sys.stdout.flush()


if __name__ == "__main__":
    main()
