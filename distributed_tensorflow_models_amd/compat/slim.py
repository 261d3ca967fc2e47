"""Functional TF-Slim facade executed eagerly on the MI355X ops (reference inception/slim/{scopes,
variables,ops,losses}.py and tf.contrib.slim).

Reference-style model code (``slim.conv2d(net, 64, [3, 3], scope='conv1')`` inside
``variable_scope``/``arg_scope`` blocks) runs unchanged: every layer call creates its variables in
the global ``VariableStore`` on first use (TF names, e.g. ``vgg_16/conv1/conv1_1/weights``) and
reuses them on later calls, so one forward pass per step both builds and executes the "graph".
Default scopes are uniquified like TF ('Conv', 'Conv_1', ...); regularizers and losses are kept
in collections (``LOSSES``, ``REGULARIZATION_LOSSES``); BatchNorm moving averages update inline.
Conv kernels are stored [K, R, S, C] and exported HWIO by the Saver (``tf_layout``).
"""
import contextlib
import functools
import math

import torch

from ..ops import elementwise as E
from ..ops import nn as F
from ..ops.lazy import as_tensor

# ---------------------------------------------------------------------------------------------
# collections / graph keys


class GraphKeys:
    GLOBAL_VARIABLES = "variables"
    TRAINABLE_VARIABLES = "trainable_variables"
    MODEL_VARIABLES = "_model_variables_"
    VARIABLES_TO_RESTORE = "_variables_to_restore_"
    MOVING_AVERAGE_VARIABLES = "moving_average_variables"
    LOSSES = "_losses"
    REGULARIZATION_LOSSES = "regularization_losses"
    UPDATE_OPS = "_update_ops_"


class VariableStore:
    def __init__(self):
        self.vars = {}
        self.collections = {}
        self.device = torch.device("cpu")
        self.scope_stack = []
        self.reuse_stack = [False]
        self.name_counts = [{}]
        self.arg_stack = [{}]
        self.training = True
        self.quant = None  # compat.quantize.QuantConfig: fake-quant training/eval graph

    def reset(self):
        self.__init__()

    def add_to_collection(self, key, value):
        self.collections.setdefault(key, []).append(value)

    def get_collection(self, key, scope=None):
        vals = self.collections.get(key, [])
        if scope:
            vals = [v for v in vals if getattr(v, "tf_name", "").startswith(scope)]
        return list(vals)


_store = VariableStore()


def get_store():
    return _store


def set_device(device):
    _store.device = torch.device(device)


def reset():
    _store.reset()


@contextlib.contextmanager
def use_store(store):
    """Run model code against a private VariableStore (one per SlimModel)."""
    global _store
    prev = _store
    _store = store
    try:
        yield store
    finally:
        _store = prev


def begin_pass():
    """Reset default-scope counters so a re-executed forward reuses the same variable names."""
    _store.scope_stack = []
    _store.name_counts = [{}]
    _store.reuse_stack = [False]
    _store.collections[GraphKeys.LOSSES] = []


def current_scope():
    return "/".join(s for s in _store.scope_stack if s)


@contextlib.contextmanager
def variable_scope(name_or_scope=None, default_name=None, values=None, reuse=None):
    """tf.variable_scope: pushes a name; with name None uses a uniquified ``default_name``."""
    if name_or_scope is None:
        name = _unique(default_name)
    else:
        name = name_or_scope
    _store.scope_stack.append(name)
    _store.reuse_stack.append(bool(reuse) or _store.reuse_stack[-1])
    _store.name_counts.append({})
    try:
        yield current_scope()
    finally:
        _store.scope_stack.pop()
        _store.reuse_stack.pop()
        _store.name_counts.pop()


name_scope = variable_scope


def _unique(base):
    counts = _store.name_counts[-1]
    n = counts.get(base, 0)
    counts[base] = n + 1
    return base if n == 0 else "%s_%d" % (base, n)


# ---------------------------------------------------------------------------------------------
# arg_scope (inception/slim/scopes.py:84-170)


def _key(fn):
    return getattr(fn, "_key_op", fn)


@contextlib.contextmanager
def arg_scope(list_ops_or_scope, **kwargs):
    if isinstance(list_ops_or_scope, dict):
        _store.arg_stack.append(list_ops_or_scope)
        try:
            yield list_ops_or_scope
        finally:
            _store.arg_stack.pop()
        return
    cur = {k: dict(v) for k, v in _store.arg_stack[-1].items()}
    for op in list_ops_or_scope:
        k = _key(op)
        if not getattr(op, "_add_arg_scope", False):
            raise ValueError("%s is not decorated with @add_arg_scope" % getattr(op, "__name__", op))
        cur.setdefault(k, {}).update(kwargs)
    _store.arg_stack.append(cur)
    try:
        yield cur
    finally:
        _store.arg_stack.pop()


def add_arg_scope(fn):
    @functools.wraps(fn)
    def wrapper(*args, **kw):
        merged = dict(_store.arg_stack[-1].get(wrapper._key_op, {}))
        merged.update(kw)  # explicit kwargs win (scopes.py:138-157)
        return fn(*args, **merged)

    wrapper._add_arg_scope = True
    wrapper._key_op = wrapper
    return wrapper


def has_arg_scope(fn):
    return getattr(fn, "_add_arg_scope", False)


# ---------------------------------------------------------------------------------------------
# variables (inception/slim/variables.py)


def _make_initializer(init, shape_tf):
    from ..models.layers import init_tensor

    def run(t):
        if init is None:
            return init_tensor(t, shape_tf, "xavier")
        if callable(init) and not isinstance(init, tuple):
            r = init(t)
            return t if r is None else r
        return init_tensor(t, shape_tf, init)
    return run


def zeros_initializer():
    return ("constant", 0.0)


def constant_initializer(v):
    return ("constant", float(v))


def truncated_normal_initializer(mean=0.0, stddev=1.0):
    return ("truncated_normal", stddev)


trunc_normal = truncated_normal_initializer


def random_normal_initializer(mean=0.0, stddev=1.0):
    return ("normal", stddev)


def xavier_initializer():
    return "xavier"


def variance_scaling_initializer(factor=2.0, mode="FAN_IN", uniform=False):
    return ("variance_scaling", (factor, mode))


class _Regularizer(tuple):
    """(kind, scale) record consumed by ``variable`` (L2 becomes coupled weight decay in the
    fused optimizer) that is also callable like slim's regularizer fns: reg(tensor) -> loss
    (inception/slim/losses.py:37-99)."""

    def __call__(self, t):
        kind, scale = self
        t = t.float()
        if kind == "l2":
            return scale * (t ** 2).sum() / 2.0
        if kind == "l1":
            return scale * t.abs().sum()
        return scale[0] * t.abs().sum() + scale[1] * (t ** 2).sum() / 2.0


def l2_regularizer(scale=1.0, scope=None):
    return _Regularizer(("l2", float(scale)))


def l1_regularizer(scale=1.0, scope=None):
    return _Regularizer(("l1", float(scale)))


def l1_l2_regularizer(scale_l1=1.0, scale_l2=1.0, scope=None):
    return _Regularizer(("l1_l2", (float(scale_l1), float(scale_l2))))


@add_arg_scope
def variable(name, shape=None, dtype=torch.float32, initializer=None, regularizer=None, trainable=True,
             collections=None, device=None, restore=True, tf_layout=None, buffer=False):
    """Create or reuse ``<scope>/<name>``; regularizers go to REGULARIZATION_LOSSES."""
    full = (current_scope() + "/" + name) if current_scope() else name
    if full in _store.vars:
        return _store.vars[full]
    shape = tuple(int(s) for s in shape)
    t = torch.empty(shape, dtype=dtype)
    shape_tf = tuple(shape[i] for i in (1, 2, 3, 0)) if tf_layout == "KRSC->HWIO" else shape
    if dtype.is_floating_point:
        _make_initializer(initializer, shape_tf)(t)
    else:
        t.zero_()
    t = t.to(device or _store.device)
    v = torch.nn.Parameter(t, requires_grad=trainable and dtype.is_floating_point and not buffer)
    v.tf_name = full
    v.tf_layout = tf_layout
    v.weight_decay = 0.0
    _store.vars[full] = v
    _store.add_to_collection(GraphKeys.GLOBAL_VARIABLES, v)
    if v.requires_grad:
        _store.add_to_collection(GraphKeys.TRAINABLE_VARIABLES, v)
    _store.add_to_collection(GraphKeys.MODEL_VARIABLES, v)
    if restore:
        _store.add_to_collection(GraphKeys.VARIABLES_TO_RESTORE, v)
    for c in collections or []:
        _store.add_to_collection(c, v)
    if regularizer is not None:
        kind, scale = regularizer
        if kind == "l2":
            v.weight_decay = scale  # applied as coupled decay by the fused optimizer
        _store.add_to_collection(GraphKeys.REGULARIZATION_LOSSES, (v, regularizer))
    return v


def global_step(device=None):
    """int64 scalar 'global_step' (inception/slim/variables.py:221-245)."""
    with _root_scope():
        return variable("global_step", (), dtype=torch.int64, trainable=False, device=device)


@contextlib.contextmanager
def _root_scope():
    saved = _store.scope_stack
    _store.scope_stack = []
    try:
        yield
    finally:
        _store.scope_stack = saved


def get_variables(scope=None, suffix=None):
    vs = _store.get_collection(GraphKeys.GLOBAL_VARIABLES, scope)
    if suffix:
        vs = [v for v in vs if v.tf_name.endswith(suffix)]
    return vs


def get_model_variables(scope=None):
    return _store.get_collection(GraphKeys.MODEL_VARIABLES, scope)


def get_variables_to_restore():
    return _store.get_collection(GraphKeys.VARIABLES_TO_RESTORE)


def trainable_variables():
    return _store.get_collection(GraphKeys.TRAINABLE_VARIABLES)


def get_variables_by_name(given_name, scope=None):
    return [v for v in get_variables(scope) if v.tf_name.split("/")[-1] == given_name]


class VariableDeviceChooser:
    """Round-robin PS placement strings (inception/slim/variables.py:175-206)."""

    def __init__(self, num_parameter_servers=0, ps_device="/job:ps", placement="CPU:0"):
        self.n, self.ps_device, self.placement = num_parameter_servers, ps_device, placement
        self.next = 0

    def __call__(self, op=None):
        if self.n > 0:
            t = self.next % self.n
            self.next += 1
            return "%s/task:%d/%s" % (self.ps_device, t, self.placement)
        return self.placement


# ---------------------------------------------------------------------------------------------
# layers


def _qvar(name, init):
    """State variable of a fake quantiser inside the current layer scope (checkpointed)."""
    return variable(name, (), initializer=("constant", float(init)), trainable=False, buffer=True)


def _qw(w):
    if _store.quant is None:
        return w
    from . import quantize as Q
    return Q.quantize_weights(w, _qvar, _store.quant)


def _qa(y):
    if _store.quant is None:
        return y
    from . import quantize as Q
    return Q.quantize_activations(as_tensor(y), _qvar, _store.quant, _store.training)


def _act(x, fn):
    if fn is None:
        return x
    if fn in (torch.relu, E.relu, "relu"):
        return E.relu(as_tensor(x))
    return fn(as_tensor(x))


relu = E.relu
relu6 = E.relu6


def _pair(v):
    return (v, v) if isinstance(v, int) else tuple(v)


@add_arg_scope
def batch_norm(inputs, decay=0.999, center=True, scale=False, epsilon=0.001, activation_fn=None,
               is_training=None, trainable=True, scope=None, reuse=None, updates_collections=None,
               param_initializers=None, fused=None, outputs_collections=None, bessel=None, data_format=None,
               zero_debias_moving_mean=False, _fold=None):
    """slim batch_norm.  ``_fold`` (internal, set by conv2d / separable_conv2d under a fake-quant
    config with ``fold_bn``): (conv_fn, weights, scale_fn) -- BatchNorm is folded into the producing
    conv's weights instead of normalising ``inputs`` (``inputs`` is then the number of channels)."""
    is_training = _store.training if is_training is None else is_training
    x = None if _fold is not None else as_tensor(inputs)
    C = inputs if _fold is not None else x.shape[-1]
    pi = param_initializers or {}
    with variable_scope(scope, "BatchNorm", reuse=reuse):
        beta = variable("beta", (C,), initializer=pi.get("beta", ("constant", 0.0)), trainable=trainable) \
            if center else None
        gamma = variable("gamma", (C,), initializer=pi.get("gamma", ("constant", 1.0)), trainable=trainable) \
            if scale else None
        mm = variable("moving_mean", (C,), initializer=("constant", 0.0), trainable=False, buffer=True,
                      collections=[GraphKeys.MOVING_AVERAGE_VARIABLES])
        mv = variable("moving_variance", (C,), initializer=("constant", 1.0), trainable=False, buffer=True,
                      collections=[GraphKeys.MOVING_AVERAGE_VARIABLES])
    mm._bn_decay = mv._bn_decay = float(decay)  # BSP BufferSync combines replicas with the layer's own decay
    if _fold is not None:  # outside the BatchNorm scope: the weight quantiser lives in the conv's scope
        return _folded_bn(_fold, gamma, beta, mm, mv, is_training, decay, epsilon, activation_fn,
                          True if bessel is None else bessel)
    relu_fused = activation_fn in (torch.relu, E.relu, "relu")
    y = F.batch_norm(x, gamma, beta, mm.data, mv.data, is_training, decay, epsilon, relu_fused, None,
                     True if bessel is None else bessel)
    return y if relu_fused else _act(y, activation_fn)


def _folded_bn(fold, gamma, beta, mm, mv, is_training, decay, epsilon, activation_fn, bessel):
    """tf.contrib.quantize fold_batch_norms (training graph without BN freeze, eval graph):
    training: the plain conv y0 = conv(x, w) gives the batch moments (gradients flow through them, as
    TF keeps that conv), the moving averages are updated from them, and the output is
    conv(x, Q(w * m)) + (beta - mean * m) with m = gamma / sqrt(var + eps) -- exactly BN(y0) when
    quantisation is off; eval: the same with the moving mean / variance."""
    conv_fn, w, scale_fn = fold[:3]
    qscope = fold[3] if len(fold) > 3 else None
    if is_training:
        y0 = as_tensor(conv_fn(w)).float()
        dims = tuple(range(y0.dim() - 1))
        mean = y0.mean(dims)
        var = y0.var(dims, unbiased=False)
        with torch.no_grad():
            n = y0.numel() // y0.shape[-1]
            uv = var * (n / max(n - 1, 1)) if bessel else var
            mm.data.sub_((mm.data - mean.detach()) * (1.0 - decay))
            mv.data.sub_((mv.data - uv.detach()) * (1.0 - decay))
    else:
        mean, var = mm.detach(), mv.detach()
    mult = torch.rsqrt(var + epsilon)
    if gamma is not None:
        mult = mult * gamma
    bias = -mean * mult
    if beta is not None:
        bias = bias + beta
    wf = scale_fn(w, mult)
    if qscope:
        with variable_scope(qscope):
            wq = _qw(wf)
    else:
        wq = _qw(wf)
    y = as_tensor(conv_fn(wq))
    y = (y.float() + bias).to(y.dtype)
    return _act(y, activation_fn)


def _fold_ok(normalizer_fn):
    q = _store.quant
    return q is not None and getattr(q, "fold_bn", False) and normalizer_fn is batch_norm


@add_arg_scope
def instance_norm(inputs, center=True, scale=True, epsilon=1e-6, activation_fn=None, param_initializers=None,
                  reuse=None, variables_collections=None, outputs_collections=None, trainable=True, data_format=None,
                  scope=None):
    """tf.contrib.layers.instance_norm: per-sample, per-channel normalisation over H, W (NHWC)."""
    x = as_tensor(inputs)
    C = x.shape[-1]
    pi = param_initializers or {}
    with variable_scope(scope, "InstanceNorm", reuse=reuse):
        beta = variable("beta", (C,), initializer=pi.get("beta", ("constant", 0.0)), trainable=trainable) \
            if center else None
        gamma = variable("gamma", (C,), initializer=pi.get("gamma", ("constant", 1.0)), trainable=trainable) \
            if scale else None
    from ..ops.activation import instance_norm as _inorm
    fuse_relu = activation_fn in (torch.relu, E.relu, "relu")
    y = _inorm(x, gamma, beta, epsilon, relu=fuse_relu)  # HIP kernel on CUDA (activation.hip)
    return y if fuse_relu else _act(y, activation_fn)


def leaky_relu(x, alpha=0.2):
    from ..ops.activation import leaky_relu as _lrelu
    return _lrelu(as_tensor(x), alpha)


def reflect_pad(x, top, bottom, left, right):
    """tf.pad(..., 'REFLECT') on NHWC (HIP gather kernel on CUDA, deterministic gather backward)."""
    from ..ops.activation import reflect_pad as _rpad
    return _rpad(as_tensor(x), top, bottom, left, right)


@add_arg_scope
def conv2d(inputs, num_outputs, kernel_size, stride=1, padding="SAME", data_format=None, rate=1,
           activation_fn=torch.relu, normalizer_fn=None, normalizer_params=None,
           weights_initializer="xavier", weights_regularizer=None, biases_initializer=("constant", 0.0),
           biases_regularizer=None, reuse=None, variables_collections=None, outputs_collections=None,
           trainable=True, scope=None):
    x = as_tensor(inputs)
    kh, kw = _pair(kernel_size)
    cin = x.shape[-1]
    with variable_scope(scope, "Conv", reuse=reuse):
        w = variable("weights", (num_outputs, kh, kw, cin), initializer=weights_initializer,
                     regularizer=weights_regularizer, trainable=trainable, tf_layout="KRSC->HWIO")
        b = None
        if normalizer_fn is None and biases_initializer is not None:
            b = variable("biases", (num_outputs,), initializer=biases_initializer, regularizer=biases_regularizer,
                         trainable=trainable)
        if normalizer_fn is not None and _fold_ok(normalizer_fn):
            fold = (lambda wt: F.conv2d(x, wt, None, stride, padding, dilation=rate), w,
                    lambda wt, m: wt * m.reshape(-1, 1, 1, 1))
            return _qa(normalizer_fn(num_outputs, activation_fn=activation_fn, _fold=fold,
                                     **(normalizer_params or {})))
        fuse = normalizer_fn is None and activation_fn in (torch.relu, E.relu, "relu")
        y = F.conv2d(x, _qw(w), b, stride, padding, relu=fuse, dilation=rate)
        if normalizer_fn is not None:
            y = normalizer_fn(y, activation_fn=activation_fn, **(normalizer_params or {}))
        elif not fuse:
            y = _act(y, activation_fn)
        return _qa(y)


convolution2d = conv2d


@add_arg_scope
def conv2d_transpose(inputs, num_outputs, kernel_size, stride=1, padding="SAME", data_format=None,
                     activation_fn=torch.relu, normalizer_fn=None, normalizer_params=None,
                     weights_initializer="xavier", weights_regularizer=None, biases_initializer=("constant", 0.0),
                     biases_regularizer=None, reuse=None, variables_collections=None, outputs_collections=None,
                     trainable=True, scope=None):
    """slim.conv2d_transpose: TF filter [kh, kw, num_outputs, in] (stored [in, kh, kw, out])."""
    x = as_tensor(inputs)
    kh, kw = _pair(kernel_size)
    cin = x.shape[-1]
    with variable_scope(scope, "Conv2d_transpose", reuse=reuse):
        w = variable("weights", (cin, kh, kw, num_outputs), initializer=weights_initializer,
                     regularizer=weights_regularizer, trainable=trainable, tf_layout="KRSC->HWIO")
        b = None
        if normalizer_fn is None and biases_initializer is not None:
            b = variable("biases", (num_outputs,), initializer=biases_initializer, regularizer=biases_regularizer,
                         trainable=trainable)
        st = stride if isinstance(stride, int) else stride[0]
        y = F.conv2d_transpose(x, w, b, st, padding)
        if normalizer_fn is not None:
            return normalizer_fn(y, activation_fn=activation_fn, **(normalizer_params or {}))
    return _act(y, activation_fn)


convolution2d_transpose = conv2d_transpose


@add_arg_scope
def separable_conv2d(inputs, num_outputs, kernel_size, depth_multiplier=1, stride=1, padding="SAME", rate=1,
                     activation_fn=torch.relu, normalizer_fn=None, normalizer_params=None,
                     weights_initializer="xavier", weights_regularizer=None, biases_initializer=("constant", 0.0),
                     trainable=True, scope=None, reuse=None, outputs_collections=None):
    from ..ops.depthwise import depthwise_conv2d
    x = as_tensor(inputs)
    kh, kw = _pair(kernel_size)
    cin = x.shape[-1]
    with variable_scope(scope, "SeparableConv2d", reuse=reuse):
        dw = variable("depthwise_weights", (kh, kw, cin, depth_multiplier), initializer=weights_initializer,
                      regularizer=weights_regularizer, trainable=trainable)
        if num_outputs is None and normalizer_fn is not None and _fold_ok(normalizer_fn):
            # depthwise-only layer (MobileNet v1): BN folded into the depthwise weights per channel
            fold = (lambda wt: depthwise_conv2d(x, wt, stride, padding, rate), dw,
                    lambda wt, m: wt * m.reshape(1, 1, cin, depth_multiplier), "depthwise_weights_q")
            return _qa(normalizer_fn(cin * depth_multiplier, activation_fn=activation_fn, _fold=fold,
                                     **(normalizer_params or {})))
        if _store.quant is not None:
            with variable_scope("depthwise_weights_q"):
                dwq = _qw(dw)
        else:
            dwq = dw
        y = depthwise_conv2d(x, dwq, stride, padding, rate)
        if num_outputs is not None and normalizer_fn is not None and _fold_ok(normalizer_fn):
            pw = variable("pointwise_weights", (num_outputs, 1, 1, cin * depth_multiplier),
                          initializer=weights_initializer, regularizer=weights_regularizer, trainable=trainable,
                          tf_layout="KRSC->HWIO")
            fold = (lambda wt: F.conv2d(y, wt, None, 1, "SAME"), pw, lambda wt, m: wt * m.reshape(-1, 1, 1, 1))
            return _qa(normalizer_fn(num_outputs, activation_fn=activation_fn, _fold=fold,
                                     **(normalizer_params or {})))
        if num_outputs is not None:
            pw = variable("pointwise_weights", (num_outputs, 1, 1, cin * depth_multiplier),
                          initializer=weights_initializer, regularizer=weights_regularizer, trainable=trainable,
                          tf_layout="KRSC->HWIO")
            y = F.conv2d(y, _qw(pw), None, 1, "SAME")
        nout = y.shape[-1]
        if normalizer_fn is not None:
            return _qa(normalizer_fn(y, activation_fn=activation_fn, **(normalizer_params or {})))
        if biases_initializer is not None:
            b = variable("biases", (nout,), initializer=biases_initializer, trainable=trainable)
            y = y + b.to(y.dtype)
        return _qa(_act(y, activation_fn))


@add_arg_scope
def fully_connected(inputs, num_outputs, activation_fn=torch.relu, normalizer_fn=None, normalizer_params=None,
                    weights_initializer="xavier", weights_regularizer=None, biases_initializer=("constant", 0.0),
                    biases_regularizer=None, reuse=None, trainable=True, scope=None, outputs_collections=None,
                    variables_collections=None):
    x = as_tensor(inputs)
    x = x.reshape(x.shape[0], -1)
    with variable_scope(scope, "fully_connected", reuse=reuse):
        w = variable("weights", (x.shape[-1], num_outputs), initializer=weights_initializer,
                     regularizer=weights_regularizer, trainable=trainable)
        b = None
        if normalizer_fn is None and biases_initializer is not None:
            b = variable("biases", (num_outputs,), initializer=biases_initializer, regularizer=biases_regularizer,
                         trainable=trainable)
        fuse = normalizer_fn is None and activation_fn in (torch.relu, E.relu, "relu")
        y = F.linear(x, _qw(w), b, relu=fuse)
        if normalizer_fn is not None:
            y = normalizer_fn(y.reshape(y.shape[0], 1, 1, -1), activation_fn=activation_fn,
                              **(normalizer_params or {}))
            return _qa(as_tensor(y).reshape(x.shape[0], -1))
        return _qa(y if fuse else _act(y, activation_fn))


fc = fully_connected


@add_arg_scope
def max_pool2d(inputs, kernel_size, stride=2, padding="VALID", scope=None, outputs_collections=None,
               data_format=None):
    return F.max_pool(inputs, _pair(kernel_size), _pair(stride), padding)


@add_arg_scope
def avg_pool2d(inputs, kernel_size, stride=2, padding="VALID", scope=None, outputs_collections=None,
               data_format=None):
    return F.avg_pool(inputs, _pair(kernel_size), _pair(stride), padding)


max_pool = max_pool2d
avg_pool = avg_pool2d


@add_arg_scope
def dropout(inputs, keep_prob=0.5, noise_shape=None, is_training=None, scope=None, outputs_collections=None):
    is_training = _store.training if is_training is None else is_training
    x = as_tensor(inputs)
    if not is_training or keep_prob >= 1.0:
        return x
    return E.dropout(x, keep_prob)


def flatten(inputs, scope=None, outputs_collections=None):
    x = as_tensor(inputs)
    return x.reshape(x.shape[0], -1)


def repeat(inputs, repetitions, layer, *args, **kwargs):
    """slim.repeat: ``layer`` applied n times inside variable scope ``scope`` (default-named
    'Repeat', 'Repeat_1', ...) with per-call scopes '<scope>_1', '<scope>_2', ... where <scope>
    falls back to the layer's __name__ (e.g. 'conv1/conv1_1', 'Repeat/block35_1')."""
    scope = kwargs.pop("scope", None)
    with variable_scope(scope, default_name="Repeat"):
        base = scope.split("/")[-1] if scope else getattr(layer, "__name__", "repeat")
        net = inputs
        for i in range(repetitions):
            net = layer(net, *args, scope="%s_%d" % (base, i + 1), **kwargs)
    return net


repeat_op = repeat


def stack(inputs, layer, stack_args, scope=None, **kwargs):
    net = inputs
    base = scope or getattr(layer, "__name__", "stack")
    with variable_scope(base):
        for i, a in enumerate(stack_args):
            a = a if isinstance(a, (list, tuple)) else (a,)
            net = layer(net, *a, scope="%s_%d" % (base.split("/")[-1], i + 1), **kwargs)
    return net


def one_hot_encoding(labels, num_classes, on_value=1.0, off_value=0.0, scope=None):
    oh = torch.full((labels.shape[0], num_classes), off_value, device=labels.device)
    oh.scatter_(1, labels.long().view(-1, 1), on_value)
    return oh


def softmax(logits, scope=None):
    return torch.softmax(as_tensor(logits).float(), -1)


# ---------------------------------------------------------------------------------------------
# losses (inception/slim/losses.py:34-174)


class losses:  # noqa: N801 (namespace like slim.losses)
    @staticmethod
    def l2_loss(tensor, weight=1.0, scope=None):
        loss = weight * (tensor.float() ** 2).sum() / 2.0
        _store.add_to_collection(GraphKeys.LOSSES, loss)
        return loss

    @staticmethod
    def l1_loss(tensor, weight=1.0, scope=None):
        loss = weight * tensor.float().abs().sum()
        _store.add_to_collection(GraphKeys.LOSSES, loss)
        return loss

    @staticmethod
    def cross_entropy_loss(logits, one_hot_labels, label_smoothing=0, weight=1.0, scope=None):
        """slim cross_entropy_loss with label smoothing y*(1-e)+e/K (losses.py:142-174)."""
        labels = one_hot_labels.argmax(-1) if one_hot_labels.dim() == 2 else one_hot_labels
        loss = weight * F.softmax_cross_entropy(as_tensor(logits), labels, label_smoothing).mean()
        _store.add_to_collection(GraphKeys.LOSSES, loss)
        return loss

    @staticmethod
    def softmax_cross_entropy(logits, onehot_labels, weights=1.0, label_smoothing=0, scope=None):
        return losses.cross_entropy_loss(logits, onehot_labels, label_smoothing, weights)

    @staticmethod
    def sparse_softmax_cross_entropy(labels, logits, weights=1.0, scope=None):
        loss = weights * F.softmax_cross_entropy(as_tensor(logits), labels, 0.0).mean()
        _store.add_to_collection(GraphKeys.LOSSES, loss)
        return loss

    @staticmethod
    def get_losses(scope=None):
        return _store.get_collection(GraphKeys.LOSSES)

    @staticmethod
    def get_regularization_losses(scope=None):
        """Materialised regularizer values (the fused optimizer applies L2 as decay instead)."""
        out = []
        for v, (kind, scale) in _store.get_collection(GraphKeys.REGULARIZATION_LOSSES):
            if kind == "l2":
                out.append(scale * (v.float() ** 2).sum() / 2.0)
            elif kind == "l1":
                out.append(scale * v.float().abs().sum())
            else:
                s1, s2 = scale
                out.append(s1 * v.float().abs().sum() + s2 * (v.float() ** 2).sum() / 2.0)
        return out

    @staticmethod
    def get_total_loss(add_regularization_losses=True):
        ls = losses.get_losses()
        if add_regularization_losses:
            ls = ls + losses.get_regularization_losses()
        return sum(ls)


def clear_losses():
    _store.collections[GraphKeys.LOSSES] = []


@contextlib.contextmanager
def training_mode(is_training):
    prev = _store.training
    _store.training = is_training
    try:
        yield
    finally:
        _store.training = prev


__all__ = [n for n in dir() if not n.startswith("_")] + ["math"]
