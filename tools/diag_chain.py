"""Diagnostic: conv+BN -> (prologue) conv+BN chain error vs. torch fp32 for several C (GPU)."""
import sys
import torch
sys.path.insert(0, ".")
from tests.test_fused_ops_gpu import _bn, _rel  # noqa: E402
from distributed_tensorflow_models_amd.ops import fused, reference as ref  # noqa: E402

DEV = "cuda"
for C in (64, 80, 96, 192, 40):
    for relu in (False, True):
        for R in (1, 3):
            torch.manual_seed(1)
            x = torch.randn(2, 10, 10, C, device=DEV).to(torch.bfloat16).float()
            w1 = (torch.randn(C, 1, 1, C, device=DEV) / C ** 0.5).to(torch.bfloat16).float()
            w2 = (torch.randn(C, R, R, C, device=DEV) / (R * R * C) ** 0.5).to(torch.bfloat16).float()
            bn1, bn2 = _bn(C), _bn(C)
            xr, w1r, w2r = (t.clone().requires_grad_() for t in (x, w1, w2))
            g1, b1 = bn1.gamma.detach().clone().requires_grad_(), bn1.beta.detach().clone().requires_grad_()
            g2, b2 = bn2.gamma.detach().clone().requires_grad_(), bn2.beta.detach().clone().requires_grad_()
            a1 = ref.batch_norm(ref.conv2d(xr, w1r), g1, b1, None, None, True, 0.9, 1e-3, relu)
            yr = ref.batch_norm(ref.conv2d(a1, w2r), g2, b2, None, None, True, 0.9, 1e-3, False)
            gy = torch.randn_like(yr).to(torch.bfloat16).float()
            yr.backward(gy)
            xk = x.to(torch.bfloat16).requires_grad_()
            w1k, w2k = w1.clone().requires_grad_(), w2.clone().requires_grad_()
            l1 = fused.conv_bn(xk, w1k, bn1, 1, "SAME", True, relu)
            l2 = fused.conv_bn(l1, w2k, bn2, 1, "SAME", True, False)
            yk = l2.materialize()
            yk.backward(gy.to(torch.bfloat16))
            torch.cuda.synchronize()
            errs = dict(y=_rel(yk, yr), dx=_rel(xk.grad, xr.grad), dw1=_rel(w1k.grad, w1r.grad),
                        dw2=_rel(w2k.grad, w2r.grad), dg1=_rel(bn1.gamma.grad, g1.grad),
                        db1=_rel(bn1.beta.grad, b1.grad), dg2=_rel(bn2.gamma.grad, g2.grad),
                        db2=_rel(bn2.beta.grad, b2.grad))
            print(C, "relu" if relu else "lin", "R%d" % R, " ".join("%s=%.4f" % kv for kv in errs.items()), flush=True)
