"""Local response normalisation (TF tf.nn.lrn semantics) - HIP kernel on GPU, torch on CPU."""
import torch

from . import _lib
from . import reference as ref
from .lazy import as_tensor


class _LRNFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, r, bias, alpha, beta):
        L = _lib.lib()
        x = x.contiguous()
        C = x.shape[-1]
        y = torch.empty_like(x)
        rc = L.dtm_lrn(_lib.ptr(x), None, _lib.ptr(y), x.numel() // C, C, r, bias, alpha, beta, 0, _lib.stream_ptr())
        if rc:
            raise RuntimeError("lrn: C > 1024 unsupported")
        ctx.save_for_backward(x)
        ctx.p = (r, bias, alpha, beta)
        return y

    @staticmethod
    def backward(ctx, dy):
        L = _lib.lib()
        (x,) = ctx.saved_tensors
        r, bias, alpha, beta = ctx.p
        C = x.shape[-1]
        dx = torch.empty_like(x)
        L.dtm_lrn(_lib.ptr(x), _lib.ptr(dy.contiguous()), _lib.ptr(dx), x.numel() // C, C, r, bias, alpha, beta, 1,
                  _lib.stream_ptr())
        return dx, None, None, None, None


def lrn(x, depth_radius=5, bias=1.0, alpha=1.0, beta=0.5):
    x = as_tensor(x)
    if not x.is_cuda:
        return ref.lrn(x, depth_radius, bias, alpha, beta)
    return _LRNFn.apply(x.to(torch.bfloat16), int(depth_radius), float(bias), float(alpha), float(beta))
