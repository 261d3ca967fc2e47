"""Training-step engine on CPU: fused-optimizer semantics (TF 1.x) and the NaN/Inf guard."""
import math

import torch

from distributed_tensorflow_models_amd.engine import TrainStep
from distributed_tensorflow_models_amd.models import nets_factory
from distributed_tensorflow_models_amd.ops.optim import FusedOptimizer


def test_nan_guard_skips_update():
    torch.manual_seed(0)
    m = nets_factory.build("lenet", 10)
    step = TrainStep(m, optimizer="momentum", lr=0.1)
    x = torch.randn(4, 28, 28, 1)
    y = torch.randint(0, 10, (4,))
    step(x, y)
    assert not step.poll_skipped()
    before = [p.detach().clone() for p in m.parameters()]
    x_bad = x.clone()
    x_bad[0, 0, 0, 0] = float("nan")
    loss = step(x_bad, y)
    assert math.isnan(float(loss))
    assert step.poll_skipped() and step.skipped == 1
    for a, p in zip(before, m.parameters()):
        assert torch.equal(a, p.detach())
    step(x, y)   # recovers on the next finite step
    assert not step.poll_skipped()


def test_tf_optimizer_semantics_cpu():
    for kind in ("sgd", "momentum", "rmsprop"):
        p = torch.nn.Parameter(torch.tensor([1.0, -2.0]))
        p.weight_decay = 0.1
        p.main_grad = torch.tensor([0.5, 0.25])
        opt = FusedOptimizer([p], kind, lr=0.1, momentum=0.9, rho=0.9, epsilon=1.0, ema_decay=0.99)
        opt.step(0.1, grad_scale=1.0)
        w0 = torch.tensor([1.0, -2.0])
        g = torch.tensor([0.5, 0.25]) + 0.1 * w0
        if kind == "sgd":
            exp = w0 - 0.1 * g
        elif kind == "momentum":
            exp = w0 - 0.1 * g                      # accum = 0*0.9 + g
        else:
            ms = 0.9 * 1.0 + 0.1 * g * g            # TF ms slot starts at 1.0
            exp = w0 - 0.1 * g / torch.sqrt(ms + 1.0)
        torch.testing.assert_close(p.detach(), exp, rtol=1e-6, atol=1e-6)
        # EMA with num_updates=0 -> decay = min(0.99, 1/10) = 0.1
        ema = opt.state[p]["ema"]
        torch.testing.assert_close(ema, w0 - (1 - 0.1) * (w0 - exp), rtol=1e-6, atol=1e-6)


import pytest  # noqa: E402


@pytest.mark.gpu
def test_nan_guard_skips_update_gpu():
    torch.manual_seed(0)
    m = nets_factory.build("resnet_v1_50", 10).cuda()
    step = TrainStep(m, optimizer="momentum", lr=0.1)
    x = torch.randn(2, 64, 64, 3, device="cuda").to(torch.bfloat16)
    y = torch.randint(0, 10, (2,), device="cuda")
    step(x, y)
    assert not step.poll_skipped()
    before = [p.detach().clone() for p in m.parameters()]
    x_bad = x.clone()
    x_bad[0, 5, 5, 0] = float("inf")
    step(x_bad, y)
    torch.cuda.synchronize()
    assert step.poll_skipped()
    assert all(torch.equal(a, p.detach()) for a, p in zip(before, m.parameters()))
