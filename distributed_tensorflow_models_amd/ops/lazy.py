"""Un-materialised BatchNorm activation (see ops.fused)."""


class LazyBN:
    """relu?(raw*scale + shift) kept as (raw, ss); ``ss`` is [4, C] (scale, shift, mean, rstd)."""

    __slots__ = ("raw", "ss", "relu")

    def __init__(self, raw, ss, relu):
        self.raw, self.ss, self.relu = raw, ss, relu

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
        return bn_apply(self.raw, self.ss, relu, residual)


def as_tensor(x):
    return x.materialize() if isinstance(x, LazyBN) else x
