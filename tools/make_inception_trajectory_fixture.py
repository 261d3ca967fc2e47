#!/usr/bin/env python3
"""CPU reference trajectories of Inception-v3 (old slim) training as the reference trains it (the fixture of
tests/test_trajectory_inception_gpu.py; config #4 of BASELINE.json).

Model and objective as /root/reference/inception/imagenet_inception_bsp.py:109-152 and
/root/reference/inception/slim/inception_model.py:54-332: 299x299 inputs, 1001 classes, BatchNorm decay 0.9997
(scale=False), L2 4e-5 on the conv / FC weights (coupled weight decay), main softmax-xent with label smoothing
0.1 plus 0.4 x the aux head's xent, RMSProp(decay 0.9, momentum 0.9, epsilon 1.0).  Dropout is disabled
(keep 1.0): its masks come from different generators on the CPU and the GPU (the dropout kernel has its own
tests).  Batch 16, 5 steps, learning rate 0.01 on a synthetic 10-pattern task (a fixed random image per class +
noise), bf16-rounded images, random-init weights (torch.manual_seed(0)).

Two CPU runs through ops/reference.py: plain fp32, and "bf16 storage" - conv weights and inputs, conv outputs,
BatchNorm outputs and average-pool outputs rounded to bf16 in forward (their gradients in backward) where the
HIP path stores bf16 tensors, everything else fp32.  Kept per run: the 5 losses, and the step-1 update of every
trainable tensor (-lr x the RMSProp-scaled gradient at w0: a whole-backward check before bf16 rounding has sent
the trajectories apart) - in full for tensors of <= 4096 elements (every BatchNorm beta, the stem conv), as a
fixed random sample of 512 elements plus the full norm for the larger ones (every conv including the merged
sibling heads, the aux head, the logits).  Usage: python tools/make_inception_trajectory_fixture.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.make_trajectory_fixture import bf16_storage as _resnet_bf16_storage, _R  # noqa: E402

STEPS, B, S, NCLS, NPAT, LR = 5, 16, 299, 1001, 10, 0.01
FULL_MAX, SAMPLE = 4096, 512
FIXTURE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "fixtures",
                       "inception_v3_299_b16")


def batches():
    g = torch.Generator().manual_seed(11)
    pat = torch.randn(NPAT, S, S, 3, generator=g)
    out = []
    for _ in range(STEPS):
        y = torch.randint(0, NPAT, (B,), generator=g)
        x = pat[y] + 0.7 * torch.randn(B, S, S, 3, generator=g)
        out.append((x.to(torch.bfloat16).float(), y + 1))  # labels 1..10 of 1001 (0 = background)
    return out


def build():
    from distributed_tensorflow_models_amd.models import nets_factory
    torch.manual_seed(0)
    return nets_factory.build("inception_v3_slim_old", num_classes=NCLS, dropout_keep_prob=1.0)


def make_step(net):
    from distributed_tensorflow_models_amd.engine import TrainStep
    return TrainStep(net, optimizer="rmsprop", lr=LR, momentum=0.9, rho=0.9, epsilon=1.0, label_smoothing=0.1,
                     aux_weight=0.4, wgrad_stream=False)


def tracked(net):
    """name -> (tensor, sample indices or None for 'all')."""
    from distributed_tensorflow_models_amd.models.layers import tf_variables
    out = {}
    for name, t, _l, trainable in tf_variables(net):
        if not trainable:
            continue
        if t.numel() <= FULL_MAX:
            out[name] = (t, None)
        else:
            g = torch.Generator().manual_seed(_stable_seed(name))
            out[name] = (t, torch.randperm(t.numel(), generator=g)[:SAMPLE])
    return out


def _stable_seed(name):
    h = 0
    for ch in name.encode():
        h = (h * 131 + ch) % (1 << 31)
    return h


def step1_update(w1, w0, idx):
    """(sampled) step-1 update and its full norm."""
    d = (w1 - w0).float().reshape(-1)
    return (d if idx is None else d[idx.to(d.device)]).cpu(), float(d.norm())


class bf16_storage(_resnet_bf16_storage):
    """ResNet fixture's emulation (conv weights / inputs / outputs and BN outputs) + average-pool outputs."""

    def __enter__(self):
        super().__enter__()
        ref = self.ref
        self.avg = ref.avg_pool

        def avg_pool(*a, **k):
            return _R.apply(self.avg(*a, **k))
        ref.avg_pool = avg_pool
        return self

    def __exit__(self, *exc):
        self.ref.avg_pool = self.avg
        super().__exit__(*exc)


def trajectory(bf16):
    import contextlib
    net = build()
    tr = tracked(net)
    w0 = {k: v.detach().clone() for k, (v, _i) in tr.items()}
    step = make_step(net)
    losses, deltas = [], {}
    with (bf16_storage() if bf16 else contextlib.nullcontext()):
        for i, (x, y) in enumerate(batches()):
            losses.append(float(step(x, y)))
            print("  step %d loss %.5f" % (i, losses[-1]), flush=True)
            if i == 0:
                for k, (v, idx) in tr.items():
                    deltas[k] = step1_update(v.detach(), w0[k], idx)
    return losses, deltas


def main():
    import numpy as np
    torch.set_num_threads(os.cpu_count() or 8)
    res = {}
    for tag, bf16 in (("fp32", False), ("emul", True)):
        print(tag, flush=True)
        res[tag] = trajectory(bf16)
    arrays = {}
    for tag, (_l, deltas) in res.items():
        for k, (d, n) in deltas.items():
            arrays["%s:%s" % (tag, k)] = d.numpy()
            arrays["%s_norm:%s" % (tag, k)] = np.array([n], np.float32)
    np.savez_compressed(FIXTURE + "_deltas.npz", **arrays)
    with open(FIXTURE + "_trajectory.json", "w") as f:
        json.dump({"model": "inception_v3_slim_old", "image": S, "batch": B, "steps": STEPS, "lr": LR,
                   "optimizer": "rmsprop(decay 0.9, momentum 0.9, eps 1.0)", "label_smoothing": 0.1,
                   "aux_weight": 0.4, "num_classes": NCLS, "dropout_keep_prob": 1.0, "device": "cpu (ops/reference.py)",
                   "losses": res["fp32"][0], "losses_bf16_storage": res["emul"][0]}, f, indent=1)
    print(res["fp32"][0])
    print(res["emul"][0])


if __name__ == "__main__":
    main()
