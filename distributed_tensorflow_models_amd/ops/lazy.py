"""Un-materialised BatchNorm activation (see ops.fused)."""


class LazyBN:
    """relu?(raw*scale + shift) kept as (raw, ss); ``ss`` is [4, C] (scale, shift, mean, rstd).

    ``unscaled``: ``raw`` comes from a training conv+BN whose backward applies the BN scale itself, so
    every consumer (all of them are fused ops: conv prologue, BN-apply, BN+ReLU+max-pool) hands back the
    gradient of the normalised pre-activation g rather than g*scale -- one elementwise multiply and, at
    a ResNet unit output, one whole gradient tensor fewer."""

    __slots__ = ("raw", "ss", "relu", "unscaled", "mat", "aslot")

    def __init__(self, raw, ss, relu, unscaled=False):
        self.raw, self.ss, self.relu, self.unscaled = raw, ss, relu, unscaled
        self.mat = None  # relu(raw*scale+shift) materialised for conv consumers (ops.fused 'mat'), shared by all
        self.aslot = None  # gradient hand-off between the conv consumers of this activation (ops.fused)

    @property
    def shape(self):
        return self.raw.shape

    @property
    def is_cuda(self):
        return self.raw.is_cuda

    @property
    def dtype(self):
        return self.raw.dtype

    @property
    def device(self):
        return self.raw.device

    def dim(self):
        return self.raw.dim()

    def materialize(self, residual=None, residual_act=None):
        from .fused import bn_apply
        relu = self.relu if residual is None else residual_act == "relu"
        return bn_apply(self.raw, self.ss, relu, residual, unscaled=self.unscaled)


class Subsampled:
    """x[:, ::s, ::s, :] (slim resnet_v1 ``subsample`` = 1x1 max-pool with stride s) kept as (src, s):
    as a block's identity residual it is read strided by the output BN-apply and its gradient is added
    strided in the other consumer's dgrad epilogue, so the subsampled tensor and its gradient are
    never stored."""

    __slots__ = ("src", "stride")

    def __init__(self, src, stride):
        self.src, self.stride = src, stride

    @property
    def shape(self):
        n, h, w, c = self.src.shape
        return (n, (h - 1) // self.stride + 1, (w - 1) // self.stride + 1, c)

    @property
    def is_cuda(self):
        return self.src.is_cuda

    def materialize(self):
        from . import nn as F
        return F.max_pool(self.src, 1, self.stride, "VALID")


def as_tensor(x):
    return x.materialize() if isinstance(x, (LazyBN, Subsampled)) else x
