#!/usr/bin/env python3
"""CPU reference trajectories of ResNet-50 v1 training (the fixture of tests/test_trajectory_gpu.py).

112x112 inputs, batch 32, 30 momentum-SGD steps on a synthetic 10-class task (a fixed random pattern
per class + noise), bf16-rounded images, random-init weights (torch.manual_seed(0)).  Two CPU runs
through ops/reference.py: plain fp32, and "bf16 storage" - conv weights, conv outputs and BatchNorm
outputs rounded to bf16 in forward (and their gradients in backward) exactly where the HIP path stores
bf16 tensors, everything else fp32.  The GPU test replays the same weights / batches through the HIP
kernels and compares per-step losses with both.  Usage: python tools/make_trajectory_fixture.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
STEPS, B, S, NCLS, LR = 30, 32, 112, 10, 0.001


def batches():
    g = torch.Generator().manual_seed(7)
    pat = torch.randn(NCLS, S, S, 3, generator=g)
    out = []
    for _ in range(STEPS):
        y = torch.randint(0, NCLS, (B,), generator=g)
        x = pat[y] + 0.7 * torch.randn(B, S, S, 3, generator=g)
        out.append((x.to(torch.bfloat16).float(), y))
    return out


def build():
    from distributed_tensorflow_models_amd.models import nets_factory
    torch.manual_seed(0)
    return nets_factory.build("resnet_v1_50", num_classes=NCLS)


class _R(torch.autograd.Function):
    """bf16 rounding in forward and of the gradient in backward (where the HIP path stores bf16)."""

    @staticmethod
    def forward(ctx, x):
        return x.to(torch.bfloat16).float()

    @staticmethod
    def backward(ctx, g):
        return g.to(torch.bfloat16).float()


class bf16_storage:
    """Patch ops.reference so conv weights / outputs and BN outputs are bf16-rounded."""

    def __enter__(self):
        from distributed_tensorflow_models_amd.ops import reference as ref
        self.ref, self.conv, self.bn = ref, ref.conv2d, ref.batch_norm

        def conv2d(x, w, bias=None, *a, **k):
            return _R.apply(self.conv(_R.apply(x), _R.apply(w), bias, *a, **k))

        def batch_norm(*a, **k):
            return _R.apply(self.bn(*a, **k))
        ref.conv2d, ref.batch_norm = conv2d, batch_norm
        return self

    def __exit__(self, *exc):
        self.ref.conv2d, self.ref.batch_norm = self.conv, self.bn


def tracked(net):
    """The tensors whose total 30-step update (w30 - w0) the fixture keeps: every BatchNorm gamma / beta
    (where a systematic BN-backward error shows first), the stem conv and the logits layer."""
    from distributed_tensorflow_models_amd.models.layers import tf_variables
    out = {}
    for name, t, _l, trainable in tf_variables(net):
        if trainable and (t.dim() == 1 or "conv1/weights" in name and "block" not in name or "logits" in name):
            out[name] = t
    return out


def trajectory(bf16, deltas=None):
    import numpy as np
    from distributed_tensorflow_models_amd.engine import TrainStep
    net = build()
    tr = tracked(net)
    w0 = {k: v.detach().clone() for k, v in tr.items()}
    step = TrainStep(net, optimizer="momentum", lr=LR, momentum=0.9)
    losses = []
    import contextlib
    with (bf16_storage() if bf16 else contextlib.nullcontext()):
        for i, (x, y) in enumerate(batches()):
            losses.append(float(step(x, y)))
            if i == 0 and deltas is not None:
                # the first update = -lr * gradient at w0: a whole-backward check before bf16 rounding has
                # had time to send the trajectories apart (by step 30 the directions are decorrelated)
                deltas.update({"step1:" + k: (v.detach() - w0[k]).float().numpy() for k, v in tr.items()})
    if deltas is not None:
        deltas.update({"norm30:" + k: np.array([float((v.detach() - w0[k]).float().norm())], np.float32)
                       for k, v in tr.items()})
    return losses


def main():
    import numpy as np
    torch.set_num_threads(os.cpu_count() or 8)
    d32, d16 = {}, {}
    fp32, b16 = trajectory(False, d32), trajectory(True, d16)
    fx = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "fixtures")
    np.savez(os.path.join(fx, "resnet50_112_b32_deltas.npz"),
             **{"fp32:" + k: v for k, v in d32.items()}, **{"emul:" + k: v for k, v in d16.items()})
    out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "fixtures",
                       "resnet50_112_b32_trajectory.json")
    with open(out, "w") as f:
        json.dump({"model": "resnet_v1_50", "image": S, "batch": B, "steps": STEPS, "lr": LR, "momentum": 0.9,
                   "num_classes": NCLS, "device": "cpu (ops/reference.py)", "losses": fp32,
                   "losses_bf16_storage": b16}, f, indent=1)
    print(fp32)
    print(b16)


if __name__ == "__main__":
    main()
