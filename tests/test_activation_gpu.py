"""HIP activation / instance-norm / reflect-pad kernels (csrc/kernels/activation.hip) against fp32
torch references, forward and backward (GPU only)."""
import pytest
import torch

from distributed_tensorflow_models_amd.ops import activation as A

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


@pytest.mark.parametrize("kind", ["relu6", "leaky_relu", "elu"])
@pytest.mark.parametrize("dtype,n", [(torch.bfloat16, 8 * 4099 + 3), (torch.float32, 100003), (torch.bfloat16, 5)])
def test_activation_kernels(kind, dtype, n):
    torch.manual_seed(0)
    x = (torch.randn(n, device=DEV) * 4).to(dtype)
    xr = x.float().clone().requires_grad_()
    yr = A._torch_act(xr, kind, 0.2)
    g = torch.randn(n, device=DEV).to(dtype)
    yr.backward(g.float())
    if kind == "relu6":  # TF Relu6Grad: g * (0 < x < 6), exclusive at both ends (torch.clamp's is inclusive)
        xf = x.float()
        xr.grad = g.float() * ((xf > 0) & (xf < 6)).float()
    xk = x.clone().requires_grad_()
    yk = A.activation(xk, kind, 0.2)
    yk.backward(g)
    tol = 1e-2 if dtype == torch.bfloat16 else 1e-6
    assert _rel(yk, yr) < tol
    # gradient through the kernel's own input (identical x): exact mask / slope
    assert _rel(xk.grad, xr.grad) < tol


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("N,H,W,C,relu,affine", [(2, 16, 16, 64, False, True), (3, 9, 7, 136, True, True),
                                                 (1, 32, 32, 32, False, False), (2, 64, 64, 128, True, True)])
def test_instance_norm_kernel(dtype, N, H, W, C, relu, affine):
    torch.manual_seed(1)
    x = (torch.randn(N, H, W, C, device=DEV) * 3 + 5).to(dtype)  # a large mean: shifted sums keep the variance
    gamma = (torch.rand(C, device=DEV) + 0.5) if affine else None
    beta = torch.randn(C, device=DEV) if affine else None
    xr = x.float().clone().requires_grad_()
    gr = gamma.clone().requires_grad_() if affine else None
    br = beta.clone().requires_grad_() if affine else None
    mean = xr.mean(dim=(1, 2), keepdim=True)
    var = xr.var(dim=(1, 2), keepdim=True, unbiased=False)
    yr = (xr - mean) * torch.rsqrt(var + 1e-6)
    if affine:
        yr = yr * gr + br
    xk = x.clone().requires_grad_()
    gk = gamma.clone().requires_grad_() if affine else None
    bk = beta.clone().requires_grad_() if affine else None
    yk = A.instance_norm(xk, gk, bk, 1e-6, relu=relu)
    dy = torch.randn_like(yr).to(dtype)
    if relu:
        mask = (yk.detach().float() > 0).float()  # the fp32 reference back-propagates through the kernel's mask
        (yr * mask).backward(dy.float())
        assert _rel(yk, torch.relu(yr)) < (2e-2 if dtype == torch.bfloat16 else 1e-5)
    else:
        yr.backward(dy.float())
        assert _rel(yk, yr) < (2e-2 if dtype == torch.bfloat16 else 1e-5)
    yk.backward(dy)
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-4
    assert _rel(xk.grad, xr.grad) < tol
    if affine:
        assert _rel(gk.grad, gr.grad) < tol and _rel(bk.grad, br.grad) < tol


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("pads,shape", [((3, 3, 3, 3), (2, 32, 32, 32)), ((1, 1, 1, 1), (1, 5, 7, 64)),
                                        ((2, 0, 1, 3), (2, 6, 5, 16))])
def test_reflect_pad_kernel(dtype, pads, shape):
    torch.manual_seed(2)
    x = torch.randn(*shape, device=DEV).to(dtype)
    t, b, l, r = pads
    xr = x.float().clone().requires_grad_()
    yr = torch.nn.functional.pad(xr.permute(0, 3, 1, 2), (l, r, t, b), mode="reflect").permute(0, 2, 3, 1)
    xk = x.clone().requires_grad_()
    yk = A.reflect_pad(xk, t, b, l, r)
    assert torch.equal(yk.float(), yr.detach())
    dy = torch.randn_like(yr).to(dtype)
    yr.backward(dy.float())
    yk.backward(dy)
    assert _rel(xk.grad, xr.grad) < (1e-2 if dtype == torch.bfloat16 else 1e-6)
