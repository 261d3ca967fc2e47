"""Small elementwise ops (ReLU/ReLU6/add/dropout) and InTopK.

On the hot path of the benchmark models these are fused into the conv / BatchNorm kernels
(epilogue ReLU, BN+residual+ReLU); the stand-alone forms below serve the remaining model-zoo
call sites.  Dropout (K15) runs the HIP kernel in ``csrc/kernels/elementwise.hip``: the keep mask is
a counter-based hash of (seed, element index), regenerated in backward, never stored.  The CPU
path evaluates the same hash with int64 tensor arithmetic, so both produce the identical mask.
"""
import ctypes

import torch

from . import _lib


def relu(x):
    return torch.relu(x)


def relu6(x):
    from .activation import relu6 as _r6  # HIP kernel on CUDA tensors (activation.hip)
    return _r6(x)


def add(x, y):
    return x + y.to(x.dtype)


def _s64(c):
    return c - (1 << 64) if c >= (1 << 63) else c


_GOLD, _M1, _M2 = _s64(0x9E3779B97F4A7C15), _s64(0xBF58476D1CE4E5B9), _s64(0x94D049BB133111EB)


def _lsr(z, s):
    """Logical right shift of int64 lanes (torch's >> is arithmetic)."""
    return (z >> s) & ((1 << (64 - s)) - 1)


def hash_u32(seed, n, device="cpu"):
    """The kernel's splitmix64-finaliser hash of (seed, i) for i < n, as int64 values in [0, 2^32)."""
    i = torch.arange(1, n + 1, dtype=torch.int64, device=device)
    z = _s64(seed % (1 << 64)) + i * _GOLD
    z = (z ^ _lsr(z, 30)) * _M1
    z = (z ^ _lsr(z, 27)) * _M2
    z = z ^ _lsr(z, 31)
    return _lsr(z, 32)


_M64 = (1 << 64) - 1


def mix_seed(seed, off):
    """Host form of the kernel's per-step stream offset (``mix_seed`` in elementwise.hip)."""
    if off == 0:
        return seed
    z = (off * 0x9E3779B97F4A7C15) & _M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
    return (seed ^ z ^ (z >> 31)) & _M64


# device int64 counter per GPU, advanced once per training step by the engine (captured into the
# hipGraph, so replays advance it too); the dropout kernel reads it at run time
_seed_off = {}


def seed_offset(device):
    device = torch.device(device)
    if device.index is None:
        device = torch.device(device.type, torch.cuda.current_device())
    t = _seed_off.get(device.index)
    if t is None:
        t = _seed_off[device.index] = torch.zeros(1, dtype=torch.int64, device=device)
    return t


def advance_seed_offset(device):
    seed_offset(device).add_(1)


def _threshold(keep):
    t = int(keep * 4294967296.0)
    return min(t, 0xFFFFFFFF)


def dropout_mask(shape, keep, seed, device="cpu"):
    n = 1
    for s in shape:
        n *= int(s)
    return (hash_u32(seed, n, device) < _threshold(keep)).reshape(shape)


def _dropout_hip(x, keep, seed):
    x = x.contiguous()
    if x.data_ptr() % 16:
        x = x.clone()
    y = torch.empty_like(x)
    dt = {torch.float32: 0, torch.bfloat16: 1}[x.dtype]
    rc = _lib.lib().dtm_dropout(_lib.ptr(x), _lib.ptr(y), x.numel(), dt, ctypes.c_float(keep),
                                ctypes.c_ulonglong(seed), _lib.ptr(seed_offset(x.device)), _lib.stream_ptr())
    if rc:
        raise RuntimeError("dtm_dropout failed (%d)" % rc)
    return y


class _DropoutFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, keep, seed):
        ctx.keep, ctx.seed = keep, seed
        if x.is_cuda:
            return _dropout_hip(x, keep, seed)
        mask = dropout_mask(x.shape, keep, seed)
        return torch.where(mask, x / keep, torch.zeros((), dtype=x.dtype))

    @staticmethod
    def backward(ctx, g):
        if g.is_cuda:
            return _dropout_hip(g, ctx.keep, ctx.seed), None, None
        mask = dropout_mask(g.shape, ctx.keep, ctx.seed)
        return torch.where(mask, g / ctx.keep, torch.zeros((), dtype=g.dtype)), None, None


_seed = [1234]


def set_base_seed(seed, rank=0):
    """Reset the dropout seed stream from the run seed and this process's rank, so every replica
    draws its own masks (each reference worker samples dropout independently) while a fixed
    (seed, rank) pair stays reproducible.  Called by the trainer and bench at start-up."""
    x = (int(seed) * 0x9E3779B97F4A7C15 + (int(rank) + 1) * 0xBF58476D1CE4E5B9) % (1 << 64)
    x ^= x >> 31
    _seed[0] = (x * 0x94D049BB133111EB) % (1 << 62)


def next_seed():
    _seed[0] = (_seed[0] * 6364136223846793005 + 1442695040888963407) % (1 << 62)
    return int(_seed[0])


def dropout(x, keep_prob, seed=None):
    """Inverted dropout: kept elements scaled by 1/keep_prob (tf.nn.dropout)."""
    if keep_prob >= 1.0:
        return x
    if x.is_cuda and x.dtype not in (torch.float32, torch.bfloat16):
        x = x.float()
    return _DropoutFn.apply(x, float(keep_prob), next_seed() if seed is None else int(seed))


def in_top_k(predictions, targets, k):
    """tf.nn.in_top_k: bool [B]; ties at the k-th value count as in, non-finite targets never do."""
    if predictions.is_cuda:
        p = predictions.contiguous()
        if p.dtype not in (torch.float32, torch.bfloat16):
            p = p.float()
        t = targets.to(torch.int32).contiguous()
        out = torch.empty(p.shape[0], dtype=torch.uint8, device=p.device)
        rc = _lib.lib().dtm_in_top_k(_lib.ptr(p), _lib.ptr(t), _lib.ptr(out), p.shape[0], p.shape[1], int(k),
                                     1 if p.dtype == torch.bfloat16 else 0, _lib.stream_ptr())
        if rc:
            raise RuntimeError("dtm_in_top_k failed (%d)" % rc)
        return out.bool()
    p = predictions.float()
    t = targets.long()
    valid = (t >= 0) & (t < p.shape[1])
    xt = p.gather(1, t.clamp(0, p.shape[1] - 1)[:, None])
    greater = (p > xt).sum(1)
    return valid & torch.isfinite(xt[:, 0]) & (greater < k)
