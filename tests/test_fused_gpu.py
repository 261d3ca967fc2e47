"""Whole small ResNet on the HIP path (fused and unfused BN) vs the torch fp32 reference on CPU."""
import copy
import os

import pytest
import torch

from distributed_tensorflow_models_amd.models.resnet_v1 import ResNetV1
from distributed_tensorflow_models_amd.ops import features
from distributed_tensorflow_models_amd.ops import fused as fused_ops

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


@pytest.mark.parametrize("fused,prologue", [("1", "auto"), ("1", "fused"), ("1", "apply"), ("0", "auto")])
@pytest.mark.parametrize("base,batch", [(16, 16), (16, 32)])
def test_small_resnet_matches_reference(fused, prologue, base, batch, monkeypatch):
    monkeypatch.setitem(features._override, "fused_bn", (fused) != "0")
    monkeypatch.setattr(fused_ops, "PROLOGUE_MODE", None if prologue == "auto" else prologue)
    torch.manual_seed(0)
    net_cpu = ResNetV1(blocks=[(base, 2, 2), (2 * base, 2, 1)], num_classes=10, scope="r")
    net_gpu = copy.deepcopy(net_cpu).cuda()
    x = torch.randn(batch, 32, 32, 3).to(torch.bfloat16).float()
    lab = torch.randint(0, 10, (batch,))
    out_c = net_cpu(x, training=True)
    loss_c = torch.nn.functional.cross_entropy(out_c.float(), lab)
    loss_c.backward()
    out_g = net_gpu(x.cuda().to(torch.bfloat16), training=True)
    loss_g = torch.nn.functional.cross_entropy(out_g.float(), lab.cuda())
    loss_g.backward()
    torch.cuda.synchronize()
    assert _rel(out_g, out_c) < 3e-2
    # A tiny random net is ill-conditioned: plain bf16 rounding of activations/grads in the CPU
    # reference already moves early-layer grads by ~30 % (a round-1 diagnostic, since removed).  So check
    # direction (cosine) for every param and tight agreement for the last layers.
    pc = dict(net_cpu.named_parameters())
    cos = {n: torch.nn.functional.cosine_similarity(p.grad.float().cpu().flatten(), pc[n].grad.float().flatten(),
                                                   dim=0).item() for n, p in net_gpu.named_parameters()}
    bad = {n: round(c, 3) for n, c in cos.items() if c < 0.85}
    assert not bad, bad
    for n, p in net_gpu.named_parameters():
        if n.startswith("logits") or "units.3.conv3.bn" in n:
            assert _rel(p.grad, pc[n].grad) < 5e-2, n
    bc = dict(net_cpu.named_buffers())
    for n, b in net_gpu.named_buffers():
        assert _rel(b, bc[n]) < 1e-2, n
