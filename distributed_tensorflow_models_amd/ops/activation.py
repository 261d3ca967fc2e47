"""ReLU6 / leaky ReLU / ELU, instance normalisation and reflect padding on the HIP path
(``csrc/kernels/activation.hip``).

Call sites: MobileNet v1/v2 ReLU6 (reference vgg/nets/mobilenet_v1.py:428-472), the DCGAN
discriminator's leaky ReLU (vgg/nets/dcgan.py:89), the CycleGAN generator's instance norm and
REFLECT padding (vgg/nets/cyclegan.py:66-117).  CUDA tensors run the kernels (hard error if the
library is missing, via ``_lib.lib()``); CPU tensors use the equivalent torch ops.
"""
import torch

from . import _lib

KIND = {"relu6": 0, "leaky_relu": 1, "elu": 2}


def _gpu(x):
    return x.is_cuda and x.dtype in (torch.bfloat16, torch.float32)


def _torch_act(x, kind, alpha):
    if kind == "relu6":
        return torch.clamp(x, 0.0, 6.0)
    if kind == "leaky_relu":
        return torch.nn.functional.leaky_relu(x, alpha)
    return torch.nn.functional.elu(x)


class _ActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, kind, alpha):
        x = x.contiguous()
        y = torch.empty_like(x)
        _lib.lib().dtm_act_fwd(_lib.ptr(x), _lib.ptr(y), x.numel(), KIND[kind], float(alpha),
                               int(x.dtype == torch.bfloat16), _lib.stream_ptr())
        ctx.save_for_backward(x)
        ctx.kind, ctx.alpha = kind, alpha
        return y

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        dy = dy.contiguous().to(x.dtype)
        dx = torch.empty_like(x)
        _lib.lib().dtm_act_bwd(_lib.ptr(dy), _lib.ptr(x), _lib.ptr(dx), x.numel(), KIND[ctx.kind], float(ctx.alpha),
                               int(x.dtype == torch.bfloat16), _lib.stream_ptr())
        return dx, None, None


def activation(x, kind, alpha=0.2):
    if _gpu(x):
        return _ActFn.apply(x, kind, alpha)
    return _torch_act(x, kind, alpha)


def relu6(x):
    return activation(x, "relu6")


def leaky_relu(x, alpha=0.2):
    return activation(x, "leaky_relu", alpha)


def elu(x):
    return activation(x, "elu")


class _InstanceNormFn(torch.autograd.Function):
    """y = act((x - mean_nc) * rsqrt(var_nc + eps) * gamma + beta), statistics per (sample, channel)
    over H, W (tf.contrib.layers.instance_norm); optional fused ReLU."""

    @staticmethod
    def forward(ctx, x, gamma, beta, eps, relu):
        x = x.contiguous()
        N, H, W, C = x.shape
        y = torch.empty_like(x)
        stats = torch.empty((N, C, 2), device=x.device, dtype=torch.float32)
        rc = _lib.lib().dtm_instnorm_fwd(_lib.ptr(x), _lib.ptr(gamma), _lib.ptr(beta), _lib.ptr(y), _lib.ptr(stats),
                                         N, H * W, C, float(eps), int(relu), int(x.dtype == torch.bfloat16),
                                         _lib.stream_ptr())
        assert rc == 0, rc
        ctx.save_for_backward(x, gamma, stats, y if relu else None)
        ctx.has_beta = beta is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, gamma, stats, y = ctx.saved_tensors
        N, H, W, C = x.shape
        dy = dy.contiguous().to(x.dtype)
        if y is not None:
            dy = torch.where(y > 0, dy, torch.zeros((), dtype=dy.dtype, device=dy.device))
        dx = torch.empty_like(x)
        sums = torch.empty((N, C, 2), device=x.device, dtype=torch.float32)
        rc = _lib.lib().dtm_instnorm_bwd(_lib.ptr(x), _lib.ptr(dy), _lib.ptr(gamma), _lib.ptr(stats), _lib.ptr(dx),
                                         _lib.ptr(sums), N, H * W, C, int(x.dtype == torch.bfloat16),
                                         _lib.stream_ptr())
        assert rc == 0, rc
        s = sums.sum(0)
        dgamma = s[:, 1] if gamma is not None else None
        dbeta = s[:, 0] if ctx.has_beta else None
        return dx, dgamma, dbeta, None, None


def instance_norm(x, gamma=None, beta=None, eps=1e-6, relu=False):
    if _gpu(x) and x.dim() == 4 and x.shape[-1] % 8 == 0:
        return _InstanceNormFn.apply(x, gamma, beta, eps, relu)
    xf = x.float()
    mean = xf.mean(dim=(1, 2), keepdim=True)
    var = xf.var(dim=(1, 2), keepdim=True, unbiased=False)
    y = (xf - mean) * torch.rsqrt(var + eps)
    if gamma is not None:
        y = y * gamma
    if beta is not None:
        y = y + beta
    if relu:
        y = torch.relu(y)
    return y.to(x.dtype)


class _ReflectPadFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, top, bottom, left, right):
        x = x.contiguous()
        N, H, W, C = x.shape
        y = torch.empty((N, H + top + bottom, W + left + right, C), device=x.device, dtype=x.dtype)
        rc = _lib.lib().dtm_reflect_pad(_lib.ptr(x), _lib.ptr(y), N, H, W, C, top, bottom, left, right,
                                        int(x.dtype == torch.bfloat16), _lib.stream_ptr())
        assert rc == 0, rc
        ctx.pads, ctx.shape = (top, bottom, left, right), (N, H, W, C)
        return y

    @staticmethod
    def backward(ctx, dy):
        N, H, W, C = ctx.shape
        top, bottom, left, right = ctx.pads
        dy = dy.contiguous()
        dx = torch.empty((N, H, W, C), device=dy.device, dtype=dy.dtype)
        rc = _lib.lib().dtm_reflect_pad_bwd(_lib.ptr(dy), _lib.ptr(dx), N, H, W, C, top, bottom, left, right,
                                            int(dy.dtype == torch.bfloat16), _lib.stream_ptr())
        assert rc == 0, rc
        return dx, None, None, None, None


def reflect_pad(x, top, bottom, left, right):
    """tf.pad(x, [[0,0],[top,bottom],[left,right],[0,0]], 'REFLECT') on NHWC."""
    if _gpu(x) and x.shape[-1] % 8 == 0 and max(top, bottom) < x.shape[1] and max(left, right) < x.shape[2]:
        return _ReflectPadFn.apply(x, top, bottom, left, right)
    y = torch.nn.functional.pad(x.permute(0, 3, 1, 2), (left, right, top, bottom), mode="reflect")
    return y.permute(0, 2, 3, 1).contiguous()
