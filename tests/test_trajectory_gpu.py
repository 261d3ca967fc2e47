"""Realistic-shape training trajectory: ResNet-50 v1 at 112x112, batch 32, 30 momentum-SGD steps through
the HIP kernels (bf16 compute, fp32 master weights / accumulation) against the CPU fp32 reference
trajectory of the same weights and batches (tests/fixtures/resnet50_112_b32_trajectory.json, written by
tools/make_trajectory_fixture.py)."""
import json
import os
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_resnet50_trajectory_matches_cpu_fp32():
    sys.path.insert(0, ROOT)
    from tools import make_trajectory_fixture as T

    from distributed_tensorflow_models_amd.engine import TrainStep
    ref = json.load(open(os.path.join(ROOT, "tests", "fixtures", "resnet50_112_b32_trajectory.json")))
    dev = torch.device("cuda", 0)
    net = T.build().to(dev)
    tr = T.tracked(net)
    w0 = {k: v.detach().clone() for k, v in tr.items()}
    step = TrainStep(net, optimizer="momentum", lr=T.LR, momentum=0.9)
    got, d1 = [], {}
    for i, (x, y) in enumerate(T.batches()):
        got.append(float(step(x.to(dev).to(torch.bfloat16), y.to(dev))))
        if i == 0:
            d1 = {k: (v.detach() - w0[k]).float().cpu() for k, v in tr.items()}
    d30 = {k: float((v.detach() - w0[k]).float().norm()) for k, v in tr.items()}
    _check_updates(d1, d30)
    fp32, emul = ref["losses"], ref["losses_bf16_storage"]

    def mrel(a, b):
        return sum(abs(u - v) / v for u, v in zip(a, b)) / len(a)
    msg = "gpu  %s\nfp32 %s\nemul %s" % tuple(["%.3f" % v for v in t] for t in (got, fp32, emul))
    # A 50-layer net at random init amplifies bf16 rounding: an exact CPU emulation of the bf16 storage
    # points (weights / conv / BN outputs) already moves the loss curve by d_emul from fp32.  The kernels
    # must stay within that noise floor: no systematic error on top of bf16 storage.
    d_gpu, d_emul = mrel(got, fp32), mrel(emul, fp32)
    assert d_gpu < 1.5 * d_emul + 5e-3, (d_gpu, d_emul, msg)
    assert max(abs(u - v) / v for u, v in zip(got, fp32)) < 0.12, msg
    assert abs(got[0] - fp32[0]) / fp32[0] < 5e-2, msg  # same weights and batch at step 0
    assert abs(sum(got) / len(got) - sum(fp32) / len(fp32)) / (sum(fp32) / len(fp32)) < 3e-2, msg


def _check_updates(d1, d30):
    """Per-tensor updates against the CPU fixtures (tests/fixtures/resnet50_112_b32_deltas.npz): every BN
    gamma / beta, the stem conv and the logits.  Step 1 (-lr x the gradient at w0, before any divergence):
    the GPU's relative error must stay within the bf16-storage emulation's own error (x1.5, + 2 %), and
    the update must not be scaled (a 5 % systematic BN-backward error fails the norm check).  Step 30: the
    typical tensor's total-update size stays within the spread that bf16 storage alone produces."""
    import numpy as np
    fx = np.load(os.path.join(ROOT, "tests", "fixtures", "resnet50_112_b32_deltas.npz"))
    bad, ratios, spread30, dev30 = [], [], [], []
    for k, g in d1.items():
        f32 = torch.from_numpy(fx["fp32:step1:" + k])
        em = torch.from_numpy(fx["emul:step1:" + k])
        n = f32.norm().item()
        if n == 0:
            continue
        e_gpu = (g - f32).norm().item() / n
        e_emu = (em - f32).norm().item() / n
        ratios.append(g.norm().item() / n)
        if e_gpu > 1.5 * e_emu + 0.02:
            bad.append("%s step-1 rel err %.4f (emulation %.4f)" % (k, e_gpu, e_emu))
        n30, e30 = float(fx["fp32:norm30:" + k][0]), float(fx["emul:norm30:" + k][0])
        spread30.append(abs(e30 - n30) / n30)
        dev30.append(abs(d30[k] - n30) / n30)
    assert not bad, "\n".join(bad[:20])
    # step 30: per tensor the update size is a single noisy sample (emulation: median 3.7 %, max 26 %), so
    # the check is on the distribution: no drift of the typical tensor's update size beyond bf16 noise
    m_gpu, m_emu = sorted(dev30)[len(dev30) // 2], sorted(spread30)[len(spread30) // 2]
    assert m_gpu < 2.0 * m_emu + 0.03, (m_gpu, m_emu)
    assert max(dev30) < 0.6, max(dev30)
    med = sorted(ratios)[len(ratios) // 2]
    assert abs(med - 1.0) < 0.03, med  # no systematic scaling (emulation: 0.999; a 5 % BN-backward error: ~0.05)
