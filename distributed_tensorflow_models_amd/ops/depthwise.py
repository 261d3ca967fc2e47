"""Depthwise conv (TF ``depthwise_conv2d`` / slim.separable_conv2d(num_outputs=None)); HIP on GPU."""
import ctypes

import torch

from . import _lib
from . import reference as ref
from .geometry import conv_geom
from .lazy import as_tensor
from .nn import _accum_param_grad


class DwArgs(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in ("N", "H", "W", "C", "M", "R", "S", "P", "Q", "stride", "ph", "pw", "dil")]


class _DepthwiseFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, a):
        L = _lib.lib()
        x = x.contiguous()
        wf = w.detach().float().contiguous()
        y = torch.empty((a.N, a.P, a.Q, a.C * a.M), device=x.device, dtype=torch.bfloat16)
        L.dtm_depthwise_fwd(_lib.ptr(x), _lib.ptr(wf), _lib.ptr(y), ctypes.byref(a), _lib.stream_ptr())
        ctx.save_for_backward(x, w)
        ctx.a = a
        return y

    @staticmethod
    def backward(ctx, dy):
        L = _lib.lib()
        x, w = ctx.saved_tensors
        a = ctx.a
        dy = dy.contiguous()
        s = _lib.stream_ptr()
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            L.dtm_depthwise_dgrad(_lib.ptr(dy), _lib.ptr(w.detach().float().contiguous()), _lib.ptr(dx),
                                  ctypes.byref(a), s)
        dw = None
        if ctx.needs_input_grad[1]:
            g = torch.zeros(w.shape, device=x.device, dtype=torch.float32)
            L.dtm_depthwise_wgrad(_lib.ptr(x), _lib.ptr(dy), _lib.ptr(g), ctypes.byref(a), s)
            dw = _accum_param_grad(w, g)
        return dx, dw, None


def depthwise_conv2d(x, w, stride=1, padding="SAME", rate=1):
    """x [N,H,W,C]; w [R,S,C,M] (TF layout, fp32 master) -> [N,P,Q,C*M]."""
    x = as_tensor(x)
    if not x.is_cuda:
        return ref.depthwise_conv2d(x, w, stride, padding, rate)
    R, S, C, M = w.shape
    g = conv_geom(tuple(x.shape), (C, R, S, C), stride, padding, rate)
    a = DwArgs(g.N, g.H, g.W, g.C, M, R, S, g.P, g.Q, g.stride, g.pad_h, g.pad_w, rate)
    return _DepthwiseFn.apply(x.to(torch.bfloat16), w, a)
