"""slim-style layer library with TensorFlow variable names (NHWC).

Every parameter carries its TF name (``tf_name``), its TF layout (conv kernels are stored
internally as [K, R, S, C] for the implicit-GEMM kernels and exported as HWIO [R, S, C, K] --
SURVEY.md §2.6 notes and §5.4), and its L2 ``weight_decay`` (slim ``l2_regularizer``: the loss
term wd*sum(w^2)/2, applied as a coupled gradient term in the fused optimizer).

Semantics follow ``tf.contrib.slim`` (reference vgg/nets/*) and the bundled old slim
(reference inception/slim/ops.py:45-476):
  conv2d = conv -> [BatchNorm | bias] -> activation;  fully_connected likewise;
  batch_norm: center=True, scale configurable, moving averages updated in training.
"""
import math

import torch
import torch.nn as nn


from ..ops import elementwise as E
from ..ops import fused
from ..ops import nn as F
from ..ops.lazy import as_tensor


def fused_enabled():
    from ..ops import features
    return features.on("fused_bn")


# ---------------------------------------------------------------------------------------------
# initialisers (TF semantics)
def _fans(shape_tf):
    if len(shape_tf) == 4:  # HWIO
        rf = shape_tf[0] * shape_tf[1]
        return shape_tf[2] * rf, shape_tf[3] * rf
    if len(shape_tf) == 2:
        return shape_tf[0], shape_tf[1]
    n = shape_tf[0] if shape_tf else 1
    return n, n


def truncated_normal_(t, std, mean=0.0):
    with torch.no_grad():
        t.normal_(0, 1)
        while True:
            bad = t.abs() > 2.0
            if not bad.any():
                break
            t[bad] = torch.randn(int(bad.sum()), dtype=t.dtype, device=t.device)
        t.mul_(std).add_(mean)
    return t


def init_tensor(t, shape_tf, init):
    """init: 'xavier' | 'variance_scaling' | ('truncated_normal', std) | ('normal', std) |
    ('constant', v) | ('uniform', a) | callable."""
    fan_in, fan_out = _fans(shape_tf)
    if callable(init):
        return init(t)
    if init == "xavier":
        lim = math.sqrt(6.0 / (fan_in + fan_out))
        with torch.no_grad():
            return t.uniform_(-lim, lim)
    if init == "variance_scaling":  # tf.contrib.layers.variance_scaling_initializer defaults
        return truncated_normal_(t, math.sqrt(1.3 * 2.0 / fan_in))
    if isinstance(init, tuple):
        kind, v = init
        if kind == "truncated_normal":
            return truncated_normal_(t, v)
        if kind == "normal":
            with torch.no_grad():
                return t.normal_(0, v)
        if kind == "constant":
            with torch.no_grad():
                return t.fill_(v)
        if kind == "uniform":
            with torch.no_grad():
                return t.uniform_(-v, v)
        if kind == "variance_scaling":
            factor, mode = v
            n = {"FAN_IN": fan_in, "FAN_OUT": fan_out, "FAN_AVG": (fan_in + fan_out) / 2.0}[mode]
            return truncated_normal_(t, math.sqrt(1.3 * factor / n))
    raise ValueError("unknown initializer %r" % (init,))


def make_param(shape, tf_name, init, tf_layout=None, weight_decay=0.0, trainable=True):
    """Create a fp32 master parameter.  tf_layout: None (same), or 'KRSC->HWIO'."""
    t = torch.empty(shape, dtype=torch.float32)
    shape_tf = tuple(shape[i] for i in (1, 2, 3, 0)) if tf_layout == "KRSC->HWIO" else tuple(shape)
    init_tensor(t, shape_tf, init)
    p = nn.Parameter(t, requires_grad=trainable)
    p.tf_name = tf_name
    p.tf_layout = tf_layout
    p.weight_decay = float(weight_decay)
    return p


def _join(scope, name):
    return name if not scope else scope + "/" + name


ACTIVATIONS = {None: None, "relu": "relu", "relu6": "relu6", "leaky_relu": "leaky_relu", "tanh": "tanh",
               "sigmoid": "sigmoid", "elu": "elu"}


def apply_activation(x, act):
    x = as_tensor(x)
    if act is None:
        return x
    if act == "relu":
        return E.relu(x)
    if act == "relu6":
        return E.relu6(x)
    if act == "leaky_relu":
        from ..ops.activation import leaky_relu
        return leaky_relu(x, 0.2)
    if act == "tanh":
        return torch.tanh(x)
    if act == "sigmoid":
        return torch.sigmoid(x)
    if act == "elu":
        from ..ops.activation import elu
        return elu(x)
    raise ValueError(act)


class Layer(nn.Module):
    def __init__(self, scope):
        super().__init__()
        self.scope = scope


# ---------------------------------------------------------------------------------------------
class BatchNorm(Layer):
    """slim.batch_norm: variables <scope>/{beta,gamma,moving_mean,moving_variance}."""

    def __init__(self, scope, channels, decay=0.999, epsilon=1e-3, center=True, scale=False, bessel=True,
                 param_initializers=None):
        super().__init__(scope)
        self.C, self.decay, self.eps, self.bessel = channels, decay, epsilon, bessel
        inits = param_initializers or {}
        self.beta = make_param((channels,), _join(scope, "beta"), inits.get("beta", ("constant", 0.0))) \
            if center else None
        self.gamma = make_param((channels,), _join(scope, "gamma"), inits.get("gamma", ("constant", 1.0))) \
            if scale else None
        self.register_buffer("moving_mean", torch.zeros(channels))
        self.register_buffer("moving_variance", torch.ones(channels))
        self.tf_buffer_names = {"moving_mean": _join(scope, "moving_mean"),
                                "moving_variance": _join(scope, "moving_variance")}

    def forward(self, x, training=True, relu=False, residual=None):
        return F.batch_norm(x, self.gamma, self.beta, self.moving_mean, self.moving_variance, training,
                            self.decay, self.eps, relu, residual, self.bessel)


class Conv2d(Layer):
    """slim.conv2d (and old-slim ops.conv2d): conv -> [BatchNorm | +bias] -> activation.

    Internal kernel layout [K, R, S, C]; TF name <scope>/weights with HWIO layout.
    """

    def __init__(self, scope, cin, cout, kernel, stride=1, padding="SAME", activation="relu", normalizer=None,
                 use_bias=None, weight_decay=0.0, init="xavier", bias_init=0.0, rate=1):
        super().__init__(scope)
        kh, kw = (kernel, kernel) if isinstance(kernel, int) else tuple(kernel)
        self.cin, self.cout, self.kh, self.kw = cin, cout, kh, kw
        self.stride, self.padding, self.rate = stride, padding, rate
        self.activation = activation
        self.weights = make_param((cout, kh, kw, cin), _join(scope, "weights"), init, "KRSC->HWIO", weight_decay)
        self.bn = None
        if normalizer is not None:
            bn_kw = dict(normalizer)
            bn_scope = bn_kw.pop("scope", "BatchNorm")
            self.bn = BatchNorm(_join(scope, bn_scope), cout, **bn_kw)
        if use_bias is None:
            use_bias = normalizer is None
        self.biases = make_param((cout,), _join(scope, "biases"), ("constant", bias_init)) if use_bias else None

    def forward(self, x, training=True, residual=None, residual_act=None):
        """residual: added after normalisation, before `residual_act` (ResNet unit output).

        On the HIP path a conv+BN returns a LazyBN (statistics from the conv epilogue, normalisation
        folded into the consumer); see ops.fused."""
        if self.bn is not None and x.is_cuda and self.rate == 1 and fused_enabled():
            relu = self.activation == "relu" and residual is None
            lazy = fused.conv_bn(x, self.weights, self.bn, self.stride, self.padding, training, relu)
            if residual is not None:
                return lazy.materialize(residual=residual, residual_act=residual_act)
            if self.activation in ("relu", None):
                return lazy
            return apply_activation(lazy.materialize(), self.activation)
        x = as_tensor(x)
        if residual is not None:
            residual = as_tensor(residual)
        fuse_relu = self.bn is None and residual is None and self.activation == "relu"
        y = F.conv2d(x, self.weights, self.biases, self.stride, self.padding, relu=fuse_relu, dilation=self.rate)
        if self.bn is not None:
            if residual is not None:
                return self.bn(y, training, relu=(residual_act == "relu"), residual=residual)
            if self.activation == "relu":
                return self.bn(y, training, relu=True)
            y = self.bn(y, training)
            return apply_activation(y, self.activation)
        if residual is not None:
            y = E.add(y, residual)
            return apply_activation(y, residual_act)
        if fuse_relu:
            return y
        return apply_activation(y, self.activation)


class FullyConnected(Layer):
    """slim.fully_connected: weights [in, out] (TF layout), biases [out]."""

    def __init__(self, scope, din, dout, activation="relu", normalizer=None, use_bias=None, weight_decay=0.0,
                 init="xavier", bias_init=0.0):
        super().__init__(scope)
        self.din, self.dout, self.activation = din, dout, activation
        self.weights = make_param((din, dout), _join(scope, "weights"), init, None, weight_decay)
        self.bn = None
        if normalizer is not None:
            bn_kw = dict(normalizer)
            bn_scope = bn_kw.pop("scope", "BatchNorm")
            self.bn = BatchNorm(_join(scope, bn_scope), dout, **bn_kw)
        if use_bias is None:
            use_bias = normalizer is None
        self.biases = make_param((dout,), _join(scope, "biases"), ("constant", bias_init)) if use_bias else None

    def forward(self, x, training=True):
        x = x.reshape(x.shape[0], -1)
        if self.bn is None:
            return F.linear(x, self.weights, self.biases, relu=self.activation == "relu") \
                if self.activation in (None, "relu") else apply_activation(F.linear(x, self.weights, self.biases),
                                                                            self.activation)
        y = F.linear(x, self.weights, None)
        y = self.bn(y.reshape(y.shape[0], 1, 1, -1), training, relu=self.activation == "relu").reshape(y.shape)
        return y if self.activation in (None, "relu") else apply_activation(y, self.activation)


class MaxPool(Layer):
    def __init__(self, scope, kernel, stride=2, padding="VALID"):
        super().__init__(scope)
        self.k, self.s, self.p = kernel, stride, padding

    def forward(self, x, training=True):
        return F.max_pool(x, self.k, self.s, self.p)


class AvgPool(Layer):
    def __init__(self, scope, kernel, stride=2, padding="VALID"):
        super().__init__(scope)
        self.k, self.s, self.p = kernel, stride, padding

    def forward(self, x, training=True):
        return F.avg_pool(x, self.k, self.s, self.p)


class Dropout(Layer):
    """slim.dropout(keep_prob): active only in training."""

    def __init__(self, scope, keep_prob=0.5):
        super().__init__(scope)
        self.keep = keep_prob

    def forward(self, x, training=True):
        if not training or self.keep >= 1.0:
            return x
        return E.dropout(x, self.keep)


def tf_variables(module):
    """Ordered list of (tf_name, tensor, tf_layout, trainable) for every variable of a model."""
    out = []
    for m in module.modules():
        for pname, p in m.named_parameters(recurse=False):
            if p is None:
                continue
            out.append((getattr(p, "tf_name", pname), p, getattr(p, "tf_layout", None), p.requires_grad))
        names = getattr(m, "tf_buffer_names", None)
        if names:
            for b, n in names.items():
                out.append((n, getattr(m, b), None, False))
    return out


def count_params(module, trainable_only=True):
    return sum(p.numel() for p in module.parameters() if p.requires_grad or not trainable_only)
