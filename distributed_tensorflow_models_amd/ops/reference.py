"""Pure-PyTorch reference implementations of every native op (NHWC).

Used (a) on CPU-only machines (unit tests, gloo multi-process plumbing), where autograd comes
from the composed torch ops, and (b) as the fp32 numerics oracle for the HIP kernels in the
GPU tests.  Semantics follow TF 1.x (asymmetric SAME padding, first-max MaxPoolGrad, avg-pool
divisor excluding padding, BN moving-average update rules).
"""
import torch
import torch.nn.functional as F

from .geometry import conv_geom, pool_geom


def _nchw(x):
    return x.permute(0, 3, 1, 2)


def _nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous()


def conv2d(x, w, bias=None, stride=1, padding="SAME", relu=False, dilation=1):
    """x [N,H,W,C], w [K,R,S,C] -> [N,P,Q,K]."""
    g = conv_geom(tuple(x.shape), tuple(w.shape), stride, padding, dilation)
    xp = _nchw(x)
    if g.pad_h or g.pad_b or g.pad_w or g.pad_r:
        xp = F.pad(xp, (g.pad_w, g.pad_r, g.pad_h, g.pad_b))
    y = F.conv2d(xp, w.permute(0, 3, 1, 2), None, g.stride, 0, dilation)
    y = y[:, :, :g.P, :g.Q]
    y = _nhwc(y)
    if bias is not None:
        y = y + bias
    if relu:
        y = torch.relu(y)
    return y


def depthwise_conv2d(x, w, stride=1, padding="SAME", dilation=1):
    """x [N,H,W,C], w [R,S,C,M] (TF depthwise layout) -> [N,P,Q,C*M]."""
    R, S, C, Mul = w.shape
    g = conv_geom(tuple(x.shape), (C, R, S, C), stride, padding, dilation)
    xp = _nchw(x)
    if g.pad_h or g.pad_b or g.pad_w or g.pad_r:
        xp = F.pad(xp, (g.pad_w, g.pad_r, g.pad_h, g.pad_b))
    wk = w.permute(2, 3, 0, 1).reshape(C * Mul, 1, R, S)
    y = F.conv2d(xp, wk, None, g.stride, 0, dilation, groups=C)
    return _nhwc(y[:, :, :g.P, :g.Q])


def conv2d_transpose(x, w, stride=2, padding="SAME", out_hw=None):
    """TF conv2d_transpose: x [N,H,W,Cin], w [R,S,Cout,Cin] -> [N,H*s,W*s,Cout] (SAME)."""
    N, H, W, Cin = x.shape
    R, S, Cout, _ = w.shape
    if out_hw is None:
        if str(padding).upper() == "SAME":
            out_hw = (H * stride, W * stride)
        else:
            out_hw = ((H - 1) * stride + R, (W - 1) * stride + S)
    # forward conv that this op is the gradient of: input out_hw, kernel [Cin? ...]
    g = conv_geom((N, out_hw[0], out_hw[1], Cout), (Cin, R, S, Cout), stride, padding)
    wk = w.permute(3, 2, 0, 1)  # [Cin, Cout, R, S] as conv weight of the forward conv (out=Cin)
    y = F.conv_transpose2d(_nchw(x), wk, None, stride, 0)
    # crop according to the forward conv's padding
    y = y[:, :, g.pad_h:g.pad_h + out_hw[0], g.pad_w:g.pad_w + out_hw[1]]
    if y.shape[2] < out_hw[0] or y.shape[3] < out_hw[1]:
        y = F.pad(y, (0, out_hw[1] - y.shape[3], 0, out_hw[0] - y.shape[2]))
    return _nhwc(y)


def batch_norm(x, gamma, beta, moving_mean, moving_var, training=True, decay=0.999, eps=1e-3, relu=False,
               residual=None, bessel=True):
    """x [..., C] (channels last).  Updates moving stats in-place when training."""
    C = x.shape[-1]
    xf = x.reshape(-1, C).float()
    if training:
        mean = xf.mean(0)
        var = xf.var(0, unbiased=False)
        if moving_mean is not None:
            with torch.no_grad():
                n = xf.shape[0]
                uvar = var * n / max(n - 1, 1) if bessel else var
                moving_mean.sub_((moving_mean - mean.detach()) * (1 - decay))
                moving_var.sub_((moving_var - uvar.detach()) * (1 - decay))
    else:
        mean, var = moving_mean, moving_var
    y = (xf - mean) * torch.rsqrt(var + eps)
    if gamma is not None:
        y = y * gamma
    if beta is not None:
        y = y + beta
    y = y.reshape(x.shape)
    if residual is not None:
        y = y + residual.float()
    if relu:
        y = torch.relu(y)
    return y.to(x.dtype) if x.dtype != torch.float32 else y


def max_pool(x, kernel, stride, padding="VALID"):
    g = pool_geom(tuple(x.shape), kernel, stride, padding)
    xp = _nchw(x)
    if g.PH or g.PB or g.PW or g.PR:
        xp = F.pad(xp, (g.PW, g.PR, g.PH, g.PB), value=float("-inf"))
    y = F.max_pool2d(xp, (g.KH, g.KW), (g.SH, g.SW))
    return _nhwc(y[:, :, :g.P, :g.Q])


def avg_pool(x, kernel, stride, padding="VALID", count_pad=False):
    g = pool_geom(tuple(x.shape), kernel, stride, padding)
    xp = _nchw(x)
    ones = torch.ones_like(xp[:, :1])
    if g.PH or g.PB or g.PW or g.PR:
        xp = F.pad(xp, (g.PW, g.PR, g.PH, g.PB))
        ones = F.pad(ones, (g.PW, g.PR, g.PH, g.PB))
    s = F.avg_pool2d(xp, (g.KH, g.KW), (g.SH, g.SW)) * (g.KH * g.KW)
    if count_pad:
        y = s / (g.KH * g.KW)
    else:
        cnt = F.avg_pool2d(ones, (g.KH, g.KW), (g.SH, g.SW)) * (g.KH * g.KW)
        y = s / cnt
    return _nhwc(y[:, :, :g.P, :g.Q])


def global_avg_pool(x):
    return x.float().mean(dim=(1, 2))


def softmax_cross_entropy(logits, labels, smoothing=0.0, row_weight=None):
    """Per-row loss; labels int64/int32 class ids."""
    lf = logits.float()
    K = lf.shape[-1]
    logp = torch.log_softmax(lf, -1)
    t = torch.full_like(lf, smoothing / K)
    t.scatter_(1, labels.long().view(-1, 1), 1.0 - smoothing + smoothing / K)
    loss = -(t * logp).sum(-1)
    if row_weight is not None:
        loss = loss * row_weight
    return loss


def lrn(x, depth_radius=5, bias=1.0, alpha=1.0, beta=0.5):
    """TF local_response_normalization over channels (NHWC):
    sqr_sum[c] = sum_{c'=c-r}^{c+r} x[c']^2;  y = x / (bias + alpha*sqr_sum)^beta."""
    xf = x.float()
    sq = (xf * xf).permute(0, 3, 1, 2)  # N C H W
    C = sq.shape[1]
    padded = F.pad(sq, (0, 0, 0, 0, depth_radius, depth_radius))
    s = sum(padded[:, i:i + C] for i in range(2 * depth_radius + 1))
    y = xf / (bias + alpha * s.permute(0, 2, 3, 1)) ** beta
    return y.to(x.dtype)
