"""Diagnostic: fused conv+BN gradient error vs. torch fp32 for several channel counts (GPU)."""
import sys
import torch
sys.path.insert(0, ".")
from tests.test_fused_ops_gpu import _bn, _rel  # noqa: E402
from distributed_tensorflow_models_amd.ops import fused, reference as ref  # noqa: E402

DEV = "cuda"
for C, K, relu in [(96, 64, True), (96, 72, True), (96, 80, True), (96, 96, True), (96, 128, True), (96, 80, False),
                   (96, 64, False)]:
    for N, HW in ((2, 12), (8, 24)):
        torch.manual_seed(0)
        x = torch.randn(N, HW, HW, C, device=DEV).to(torch.bfloat16).float()
        w = (torch.randn(K, 1, 1, C, device=DEV) / C ** 0.5).to(torch.bfloat16).float()
        bn = _bn(K)
        xr, wr = x.clone().requires_grad_(), w.clone().requires_grad_()
        gr, br = bn.gamma.detach().clone().requires_grad_(), bn.beta.detach().clone().requires_grad_()
        yr = ref.batch_norm(ref.conv2d(xr, wr, None, 1, "SAME"), gr, br, None, None, True, 0.9, 1e-3, relu)
        gy = torch.randn_like(yr).to(torch.bfloat16).float()
        yr.backward(gy)
        xk = x.to(torch.bfloat16).requires_grad_()
        wk = w.clone().requires_grad_()
        yk = fused.conv_bn(xk, wk, bn, 1, "SAME", True, relu).materialize()
        yk.backward(gy.to(torch.bfloat16))
        torch.cuda.synchronize()
        # dbeta directly = sum(g * mask) computed from our own y
        m = (yk.float() > 0).float() if relu else torch.ones_like(yk.float())
        dbeta_own = (gy * m).sum((0, 1, 2))
        print(C, K, relu, N, HW, {k: round(v, 4) for k, v in dict(
            y=_rel(yk, yr), dx=_rel(xk.grad, xr.grad), dw=_rel(wk.grad, wr.grad),
            dgamma=_rel(bn.gamma.grad, gr.grad), dbeta=_rel(bn.beta.grad, br.grad),
            dbeta_vs_own_mask=_rel(bn.beta.grad, dbeta_own)).items()}, flush=True)
