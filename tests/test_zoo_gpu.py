"""GPU checks of the wider model zoo: conv2d_transpose numerics against the torch fp32 oracle, and
every zoo family (Inception-v4 / Inception-ResNet-v2, NASNet / PNASNet cells, MobileNets, GANs)
running forward + backward on the HIP kernels, with inference logits matching the CPU oracle."""
import copy

import pytest
import torch

from distributed_tensorflow_models_amd.compat import slim
from distributed_tensorflow_models_amd.models import gans, nets_factory
from distributed_tensorflow_models_amd.ops import nn as dnn
from distributed_tensorflow_models_amd.ops import reference as ref
from distributed_tensorflow_models_amd.ops import features

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


@pytest.mark.parametrize("N,H,Cx,Cy,R,stride,pad", [
    (2, 8, 64, 32, 4, 2, "SAME"), (2, 7, 32, 64, 3, 2, "VALID"), (3, 1, 64, 128, 4, 1, "VALID"),
    (2, 16, 64, 3, 4, 2, "SAME"), (2, 9, 24, 16, 3, 1, "SAME"), (1, 5, 20, 8, 3, 2, "SAME")])
def test_conv2d_transpose(N, H, Cx, Cy, R, stride, pad):
    torch.manual_seed(0)
    x = torch.randn(N, H, H, Cx, device=DEV).to(torch.bfloat16).float()
    w = (torch.randn(Cx, R, R, Cy, device=DEV) / (R * R * Cx) ** 0.5).to(torch.bfloat16).float()
    # fp32 reference on the CPU: MIOpen's own find step for the odd small shapes here ran a solver that faulted the
    # GPU (illegal address inside MIOpen's EvaluateInvokers, round-4 final suite) - the reference must not do that
    xr, wr = x.cpu().clone().requires_grad_(), w.cpu().clone().requires_grad_()
    yr = ref.conv2d_transpose(xr, wr.permute(1, 2, 3, 0), stride, pad)
    gy = torch.randn_like(yr).to(torch.bfloat16).float()
    yr.backward(gy)
    xk = x.to(torch.bfloat16).requires_grad_()
    wk = w.clone().requires_grad_()
    yk = dnn.conv2d_transpose(xk, wk, None, stride, pad)
    assert yk.shape == yr.shape
    yk.backward(gy.to(DEV, torch.bfloat16))
    torch.cuda.synchronize()
    errs = dict(y=_rel(yk, yr), dx=_rel(xk.grad, xr.grad), dw=_rel(wk.grad, wr.grad))
    assert all(v < 1.5e-2 for v in errs.values()), errs


@pytest.mark.parametrize("N,H,C,M,R,stride,pad", [
    (2, 14, 32, 1, 3, 1, "SAME"), (2, 15, 64, 1, 3, 2, "SAME"), (2, 16, 11, 1, 5, 2, "SAME"),
    (1, 21, 96, 1, 7, 1, "SAME"), (2, 12, 3, 8, 7, 2, "SAME"), (2, 9, 16, 2, 3, 1, "VALID")])
def test_depthwise_conv2d(N, H, C, M, R, stride, pad):
    from distributed_tensorflow_models_amd.ops.depthwise import depthwise_conv2d
    torch.manual_seed(0)
    x = torch.randn(N, H, H, C, device=DEV).to(torch.bfloat16).float()
    w = (torch.randn(R, R, C, M, device=DEV) / R).to(torch.bfloat16).float()
    xr, wr = x.cpu().clone().requires_grad_(), w.cpu().clone().requires_grad_()  # (CPU fp32 reference: no MIOpen)
    yr = ref.depthwise_conv2d(xr, wr, stride, pad)
    gy = torch.randn_like(yr).to(torch.bfloat16).float()
    yr.backward(gy)
    xk = x.to(torch.bfloat16).requires_grad_()
    wk = w.clone().requires_grad_()
    yk = depthwise_conv2d(xk, wk, stride, pad)
    yk.backward(gy.to(DEV, torch.bfloat16))
    torch.cuda.synchronize()
    errs = dict(y=_rel(yk, yr), dx=_rel(xk.grad, xr.grad), dw=_rel(wk.grad, wr.grad))
    assert all(v < 1.5e-2 for v in errs.values()), errs


ZOO = [("inception_v4", 299, 1001, 2), ("inception_resnet_v2", 299, 1001, 2), ("nasnet_cifar", 32, 10, 4),
       ("nasnet_mobile", 224, 1001, 2), ("mobilenet_v1", 224, 1001, 2), ("mobilenet_v2", 224, 1001, 2),
       ("inception_v1", 224, 1001, 2), ("inception_v2", 224, 1001, 2), ("resnet_v2_50", 224, 1001, 2)]


@pytest.mark.parametrize("name,size,nc,B", ZOO)
def test_zoo_train_step_and_oracle(name, size, nc, B):
    torch.manual_seed(0)
    cpu = nets_factory.build(name, nc)
    gpu = copy.deepcopy(cpu).to(DEV)
    x = torch.randn(B, size, size, 3)
    with torch.no_grad():
        ref_logits = cpu(x, training=False)
        got = gpu(x.to(DEV, torch.bfloat16), training=False)
        # random-init nets in inference mode can be chaotic (MobileNets: a 0.4 % input perturbation
        # moves the fp32 logits by ~13 %, a round-4 diagnostic); bound the bf16 HIP result by the
        # oracle's own sensitivity to a bf16-sized perturbation
        g = torch.Generator().manual_seed(1)
        sens = _rel(cpu(x * (1 + 0.004 * torch.randn(x.shape, generator=g)), training=False), ref_logits)
    assert _rel(got, ref_logits) < max(6e-2, 3 * sens)
    y = torch.randint(0, nc, (B,), device=DEV)
    out = gpu(x.to(DEV, torch.bfloat16), training=True)
    logits = out[0] if isinstance(out, tuple) else out
    loss = dnn.softmax_cross_entropy(logits, y).mean()
    if isinstance(out, tuple):
        loss = loss + 0.4 * dnn.softmax_cross_entropy(out[1], y).mean()
    loss.backward()
    torch.cuda.synchronize()
    assert torch.isfinite(loss)
    grads = [p.grad for p in gpu.parameters() if p.requires_grad and p.grad is not None]
    assert len(grads) > 0.9 * sum(1 for p in gpu.parameters() if p.requires_grad)
    assert all(torch.isfinite(g).all() for g in grads)


@pytest.mark.parametrize("name", ["resnet_v1_50", "resnet_v2_50"])
def test_atrous_resnet_output_stride_16(name):
    """Dense-prediction mode (output_stride 16: block4 runs with rate 2 on the dilated-conv path,
    mixed with the fused conv+BN units) against the fp32 oracle, then one backward."""
    torch.manual_seed(0)
    cpu = nets_factory.build(name, 10, output_stride=16, global_pool=False, spatial_squeeze=False)
    gpu = copy.deepcopy(cpu).to(DEV)
    x = torch.randn(2, 129, 129, 3)
    with torch.no_grad():
        want = cpu(x, training=False)
        got = gpu(x.to(DEV, torch.bfloat16), training=False)
    assert list(got.shape) == [2, 9, 9, 10] == list(want.shape)
    assert _rel(got, want) < 6e-2
    out = gpu(x.to(DEV, torch.bfloat16), training=True)
    out.float().square().mean().backward()
    torch.cuda.synchronize()
    grads = [p.grad for p in gpu.parameters() if p.requires_grad and p.grad is not None]
    assert len(grads) > 0.9 * sum(1 for p in gpu.parameters() if p.requires_grad)
    assert all(torch.isfinite(g).all() for g in grads)


def _gan(fn, *a, **k):
    st = slim.VariableStore()
    st.device = DEV
    with slim.use_store(st):
        slim.begin_pass()
        out = fn(*a, **k)
    return out, st


@pytest.mark.parametrize("kind", ["dcgan", "cyclegan", "pix2pix"])
def test_gans_forward_backward(kind):
    torch.manual_seed(0)
    if kind == "dcgan":
        (img, _), st = _gan(gans.dcgan_generator, torch.randn(4, 64, device=DEV), depth=32, final_size=32)
        (d, _), _ = _gan(gans.dcgan_discriminator, img, depth=32)
        loss = d.float().mean()
    elif kind == "cyclegan":
        x = torch.randn(2, 64, 64, 3, device=DEV).to(torch.bfloat16)
        (y, _), st = _gan(gans.cyclegan_generator_resnet, x)
        assert y.shape == x.shape
        loss = y.float().square().mean()
    else:
        x = torch.randn(2, 64, 64, 3, device=DEV).to(torch.bfloat16)

        def fn(t):
            with gans.pix2pix_arg_scope():
                return gans.pix2pix_generator(t, 3, blocks=[(64, 0.5), (128, 0.5), (256, 0)],
                                              upsample_method="conv2d_transpose")
        (y, _), st = _gan(fn, x)
        assert list(y.shape) == [2, 64, 64, 3]
        loss = y.float().square().mean()
    loss.backward()
    torch.cuda.synchronize()
    params = [v for v in st.vars.values() if v.requires_grad]
    assert all(v.grad is not None and torch.isfinite(v.grad).all() for v in params)


@pytest.mark.parametrize("Cs", [(64, 96, 32, 48), (320, 384, 384, 192), (8, 16)])
def test_zero_copy_concat_exact(Cs):
    """concat_channels of LazyBN parts (+ a plain tensor part) == torch.cat of the materialised parts,
    bit for bit, forward and backward (raw-input gradient and the BN-statistics gradient)."""
    from distributed_tensorflow_models_amd.ops.fused import bn_apply, concat_channels
    from distributed_tensorflow_models_amd.ops.lazy import LazyBN
    torch.manual_seed(0)
    N, H, W = 3, 9, 7
    raws = [torch.randn(N, H, W, c, device=DEV).to(torch.bfloat16) for c in Cs]
    sss = [torch.cat([torch.rand(1, c, device=DEV) + 0.5, torch.randn(1, c, device=DEV) * 0.3,
                      torch.randn(2, c, device=DEV)]) for c in Cs]
    plain = torch.randn(N, H, W, 24, device=DEV).to(torch.bfloat16)
    dout = torch.randn(N, H, W, sum(Cs) + 24, device=DEV).to(torch.bfloat16)
    outs = []
    for zero_copy in (True, False):
        rs = [r.clone().requires_grad_() for r in raws]
        ss = [x.clone().requires_grad_() for x in sss]
        pl = plain.clone().requires_grad_()
        lz = [LazyBN(r, s, True, unscaled=True) for r, s in zip(rs, ss)]
        if zero_copy:
            y = concat_channels(lz + [pl])
        else:
            y = torch.cat([bn_apply(r, s, True, None, unscaled=True) for r, s in zip(rs, ss)] + [pl], -1)
        y.backward(dout)
        outs.append((y.detach(), [r.grad for r in rs], [s.grad for s in ss], pl.grad))
    (ya, ra, sa, pa), (yb, rb, sb, pb) = outs
    assert torch.equal(ya, yb) and torch.equal(pa, pb)
    for a, b in zip(ra, rb):
        assert torch.equal(a, b)
    for a, b in zip(sa, sb):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("Cs", [(64, 96, 32, 48), (320, 384, 384, 192), (192, 192, 192, 192), (8, 16)])
def test_zero_copy_concat_one_launch(monkeypatch, Cs):
    """All-BN concats take the one-launch multi-part kernels (every part's BN-apply, then every part's
    backward + one reduction of the dss rows): bit-identical output / masks / input gradients to the
    per-part launches and torch.cat, the statistics gradients equal up to summation order."""
    from distributed_tensorflow_models_amd.ops.fused import bn_apply, concat_channels
    from distributed_tensorflow_models_amd.ops.lazy import LazyBN
    torch.manual_seed(0)
    N, H, W = 4, 9, 7
    raws = [torch.randn(N, H, W, c, device=DEV).to(torch.bfloat16) for c in Cs]
    sss = [torch.cat([torch.rand(1, c, device=DEV) + 0.5, torch.randn(1, c, device=DEV) * 0.3,
                      torch.randn(2, c, device=DEV)]) for c in Cs]
    dout = torch.randn(N, H, W, sum(Cs), device=DEV).to(torch.bfloat16)
    outs = []
    for mode in ("multi", "parts", "cat"):
        monkeypatch.setitem(features._override, "cat_multi", mode != "parts")
        rs = [r.clone().requires_grad_() for r in raws]
        ss = [x.clone().requires_grad_() for x in sss]
        lz = [LazyBN(r, s, True, unscaled=(i % 2 == 0)) for i, (r, s) in enumerate(zip(rs, ss))]
        if mode == "cat":
            y = torch.cat([bn_apply(r, s, True, None, unscaled=(i % 2 == 0)) for i, (r, s) in enumerate(zip(rs, ss))],
                          -1)
        else:
            y = concat_channels(lz)
        y.backward(dout)
        torch.cuda.synchronize()
        outs.append((y.detach(), [r.grad for r in rs], [s.grad for s in ss]))
    (ya, ra, sa), (yb, rb, sb), (yc, rc, sc) = outs
    assert torch.equal(ya, yb) and torch.equal(ya, yc)
    for a, b, c in zip(ra, rb, rc):
        assert torch.equal(a, b) and torch.equal(a, c)
    for a, b, c in zip(sa, sb, sc):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-4)
        torch.testing.assert_close(a, c, rtol=1e-5, atol=1e-4)


def test_inception_zero_copy_concat_matches_torch_cat(monkeypatch):
    """Old-slim Inception-v3 with branch outputs BN-applied straight into their concat slices (and
    their gradients read in place) vs the same model through torch.cat of materialised branches.
    Inference-mode BN (moving statistics) keeps the comparison deterministic: in training mode the
    fp32-atomic batch statistics differ in the last bit between any two runs with different
    allocation histories (even torch.cat vs torch.cat + clone), and a batch-2 BN network amplifies
    that chaotically (a round-4 diagnostic); the training-mode concat itself is checked bit for bit
    by test_zero_copy_concat_exact."""
    from distributed_tensorflow_models_amd.models import inception_v3_slim as iv3
    from distributed_tensorflow_models_amd.ops.lazy import as_tensor

    def run(zero_copy):
        if not zero_copy:
            monkeypatch.setattr(iv3, "concat_channels", lambda parts: torch.cat([as_tensor(p) for p in parts], -1))
        torch.manual_seed(0)
        net = nets_factory.build("inception_v3_slim_old", num_classes=11).to(DEV)
        g = torch.Generator().manual_seed(1)
        x = torch.randn(2, 299, 299, 3, generator=g).to(DEV, torch.bfloat16)
        logits = net(x, training=False)
        logits.float().square().mean().backward()
        torch.cuda.synchronize()
        monkeypatch.undo()
        grads = torch.cat([p.grad.float().reshape(-1) for p in net.parameters() if p.grad is not None])
        return logits.float(), grads

    la, ga = run(True)
    lb, gb = run(False)
    assert torch.equal(la, lb)
    assert _rel(ga, gb) < 1e-3


@pytest.mark.parametrize("pool", ["avg", "max"])
def test_pool_joins_shared_input_grad_handoff(pool):
    """A pooling branch reading a tensor shared with fused conv consumers hands its input gradient
    to the last conv's dgrad epilogue (grad_handoff=True): same x.grad as autograd's add."""
    from distributed_tensorflow_models_amd.models.layers import Conv2d
    from distributed_tensorflow_models_amd.ops import nn as F
    from distributed_tensorflow_models_amd.ops.lazy import as_tensor
    torch.manual_seed(0)
    bn = dict(decay=0.9997, epsilon=1e-3, scale=False, bessel=False)
    convs = [Conv2d("c%d" % i, 64, 32, k, 1, "SAME", "relu", dict(bn), False, 0.0, ("truncated_normal", 0.1)).to(DEV)
             for i, k in enumerate((1, 3))]
    x0 = torch.randn(4, 17, 17, 64, device=DEV).to(torch.bfloat16)
    grads = []
    for handoff in (True, False):
        x = x0.clone().requires_grad_()
        outs = [as_tensor(c(x, True)) for c in convs]
        p = (F.avg_pool(x, 3, 1, "SAME", grad_handoff=handoff) if pool == "avg"
             else F.max_pool(x, 3, 1, "SAME", grad_handoff=handoff))
        loss = sum(o.float().square().mean() for o in outs) + p.float().square().mean() * 3
        loss.backward()
        grads.append(x.grad.float())
    assert _rel(grads[0], grads[1]) < 1e-2


@pytest.mark.parametrize("aux_in_loss", [True, False])
@pytest.mark.parametrize("fused_bn", [True, False])
def test_aux_pool_tail_adds_into_main_gradient(aux_in_loss, fused_bn):
    """Inception's aux-head pool as a tail consumer (avg_pool grad_tail=True, recorded before the block's slot
    consumers): its gradient is added in place into the one the last consumer returns - same x.grad as autograd's
    add; and with the aux output left out of the loss (its backward never runs) x.grad is exactly the no-tail one.
    With fused_bn off (generic conv consumers, the pool the only slot consumer) the tail must stay off and x.grad
    still include the aux gradient (it was added into a stale tensor and lost)."""
    from distributed_tensorflow_models_amd.models.layers import Conv2d
    from distributed_tensorflow_models_amd.ops import features
    from distributed_tensorflow_models_amd.ops import nn as F
    from distributed_tensorflow_models_amd.ops.lazy import as_tensor
    torch.manual_seed(0)
    bn = dict(decay=0.9997, epsilon=1e-3, scale=False, bessel=False)
    convs = [Conv2d("c%d" % i, 64, 32, k, 1, "SAME", "relu", dict(bn), False, 0.0, ("truncated_normal", 0.1)).to(DEV)
             for i, k in enumerate((1, 3))]
    x0 = torch.randn(4, 17, 17, 64, device=DEV).to(torch.bfloat16)
    grads, fused = [], []
    for tail in (True, False):
        with features.override(pool_tail=tail, fused_bn=fused_bn):
            x = x0.clone().requires_grad_()
            before = F.TAIL_FUSED[0]
            aux = F.avg_pool(x, 5, 3, "VALID", grad_tail=True)
            outs = [as_tensor(c(x, True)) for c in convs]
            p = F.max_pool(x, 3, 2, "VALID", grad_handoff=True)
            loss = sum(o.float().square().mean() for o in outs) + p.float().square().mean() * 3
            if aux_in_loss:
                loss = loss + aux.float().square().mean() * 5
            loss.backward()
            torch.cuda.synchronize()
            grads.append(x.grad.float())
            fused.append(F.TAIL_FUSED[0] - before)
    assert fused == [1 if (aux_in_loss and fused_bn) else 0, 0], fused
    if aux_in_loss:
        assert _rel(grads[0], grads[1]) < 1e-2
    else:
        assert torch.equal(grads[0], grads[1])


@pytest.mark.parametrize("C,K,H", [(288, 64, 35), (768, 192, 17), (2048, 192, 8)])
def test_pool_branch_commuted(C, K, H):
    """Inception pool branch avg_pool(3x3/1 SAME) -> 1x1 conv -> BN+ReLU computed as 1x1 conv -> avg_pool ->
    BN (fused.conv_avgpool_bn): output, input / weight / BN-parameter gradients and moving statistics are
    as close to the fp32 reference (original order) as the bf16 original-order path is (training-mode
    batch statistics; the residual difference is bf16 rounding of different intermediates and the ReLU
    mask flips it causes)."""
    from distributed_tensorflow_models_amd.models.layers import Conv2d
    from distributed_tensorflow_models_amd.ops import fused
    from distributed_tensorflow_models_amd.ops import nn as F
    from distributed_tensorflow_models_amd.ops import reference as ref
    bn = dict(decay=0.9997, epsilon=1e-3, scale=False, bessel=False)
    torch.manual_seed(0)
    x0 = torch.randn(8, H, H, C, device=DEV).to(torch.bfloat16)
    gy0 = torch.randn(8, H, H, K, device=DEV).to(torch.bfloat16)
    res = []
    for mode in ("ref", "orig", "commute"):
        torch.manual_seed(0)
        conv = Conv2d("pool_conv", C, K, 1, 1, "SAME", "relu", dict(bn), False, 0.0, ("truncated_normal", 0.1)).to(DEV)
        if mode == "ref":
            x = x0.float().requires_grad_()
            w = conv.weights.detach().float().requires_grad_()
            beta = conv.bn.beta.detach().clone().requires_grad_()
            mm, mv = conv.bn.moving_mean.clone(), conv.bn.moving_variance.clone()
            y = ref.batch_norm(ref.conv2d(ref.avg_pool(x, 3, 1, "SAME"), w, None, 1, "SAME"), None, beta, mm, mv,
                               True, 0.9997, 1e-3, True, None, False)
            y.backward(gy0.float())
            res.append((y, x.grad, w.grad, beta.grad, mm, mv))
            continue
        x = x0.clone().requires_grad_()
        if mode == "commute":
            lz = fused.conv_avgpool_bn(x, conv.weights, conv.bn, True, relu=True)
        else:
            lz = conv(F.avg_pool(x, 3, 1, "SAME"), True)
        y = lz.materialize()
        y.backward(gy0)
        torch.cuda.synchronize()
        res.append((y.float(), x.grad.float(), conv.weights.grad.float(), conv.bn.beta.grad.float(),
                    conv.bn.moving_mean.clone(), conv.bn.moving_variance.clone()))
    for r, o, c in zip(*res):
        eo, ec = _rel(o, r), _rel(c, r)
        assert ec < max(1.5 * eo, 2e-2), (eo, ec)
