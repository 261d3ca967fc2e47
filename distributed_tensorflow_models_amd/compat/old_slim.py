"""The bundled *old* TF-Slim API (reference inception/slim/{ops,scopes,variables,losses}.py,
SURVEY.md §2.7 C40-C44) on top of the eager slim facade in ``compat.slim``.

Reference code written against ``from inception.slim import slim`` (``slim.ops.conv2d(net, 64, [3, 3],
stddev=0.1, batch_norm_params=..., scope='conv0')``, ``slim.scopes.arg_scope``, ``slim.variables``,
``slim.losses``) keeps its call shapes and variable names:

* ``ops.conv2d`` / ``ops.fc``: default scopes 'Conv' / 'FC' (uniquified), truncated-normal weights
  (``stddev``), L2 ``weight_decay`` on the weights only, either ``biases`` (init ``bias``) or a
  BatchNorm built from ``batch_norm_params`` inside the layer scope ('Conv/BatchNorm/beta');
* ``ops.batch_norm``: center=True, scale=False, eps 1e-3, decay 0.999, *biased* batch moments
  (tf.nn.moments, ops.py:117-124); the two moving-average updates are recorded in
  ``UPDATE_OPS_COLLECTION`` as '<scope>/AssignMovingAvg', '<scope>/AssignMovingAvg_1' (they run
  inline, eagerly, on the HIP BN kernels);
* ``ops.max_pool`` / ``ops.avg_pool``: default stride 2, 'VALID'; ``ops.dropout`` is the identity
  when not training; ``ops.repeat_op`` scopes 'conv1/Conv', 'conv1/Conv_1', ...
All compute goes through the same MI355X ops as the rest of the framework (``ops.nn``).
"""
import types

import torch

from . import slim as _s
from ..ops import elementwise as E
from ..ops import nn as F
from ..ops.lazy import as_tensor

UPDATE_OPS_COLLECTION = _s.GraphKeys.UPDATE_OPS            # '_update_ops_'
MODEL_VARIABLES = _s.GraphKeys.MODEL_VARIABLES            # '_model_variables_'
VARIABLES_TO_RESTORE = _s.GraphKeys.VARIABLES_TO_RESTORE  # '_variables_to_restore_'
LOSSES_COLLECTION = _s.GraphKeys.LOSSES                   # '_losses'


def _pair(v):
    return (int(v), int(v)) if isinstance(v, int) else tuple(int(i) for i in v)


def _activate(y, activation):
    if activation is None:
        return y
    if activation in (torch.relu, E.relu, "relu"):
        return E.relu(as_tensor(y))
    return activation(as_tensor(y))


# ---------------------------------------------------------------------------------------------
# ops.py
@_s.add_arg_scope
def batch_norm(inputs, decay=0.999, center=True, scale=False, epsilon=0.001, moving_vars="moving_vars",
               activation=None, is_training=True, trainable=True, restore=True, scope=None, reuse=None):
    """ops.batch_norm (inception/slim/ops.py:45-135)."""
    x = as_tensor(inputs)
    C = x.shape[-1]
    with _s.variable_scope(scope, "BatchNorm", reuse=reuse) as sc:
        beta = _s.variable("beta", (C,), initializer=("constant", 0.0), trainable=trainable, restore=restore) \
            if center else None
        gamma = _s.variable("gamma", (C,), initializer=("constant", 1.0), trainable=trainable, restore=restore) \
            if scale else None
        mm = _s.variable("moving_mean", (C,), initializer=("constant", 0.0), trainable=False, restore=restore,
                         buffer=True, collections=[moving_vars, _s.GraphKeys.MOVING_AVERAGE_VARIABLES])
        mv = _s.variable("moving_variance", (C,), initializer=("constant", 1.0), trainable=False, restore=restore,
                         buffer=True, collections=[moving_vars, _s.GraphKeys.MOVING_AVERAGE_VARIABLES])
        if is_training:
            store = _s.get_store()
            for suffix in ("AssignMovingAvg", "AssignMovingAvg_1"):
                name = sc + "/" + suffix
                if name not in store.collections.get(UPDATE_OPS_COLLECTION, []):
                    store.add_to_collection(UPDATE_OPS_COLLECTION, name)
    mm._bn_decay = mv._bn_decay = float(decay)  # BSP BufferSync combines replicas with the layer's own decay
    relu = activation in (torch.relu, E.relu, "relu")
    y = F.batch_norm(x, gamma, beta, mm.data, mv.data, bool(is_training), decay, epsilon, relu, None, False)
    return y if relu else _activate(y, activation)


def _bn_or_bias(y, num_out, bias, batch_norm_params, is_training, trainable, restore):
    if batch_norm_params is not None:
        with _s.arg_scope([batch_norm], is_training=is_training, trainable=trainable, restore=restore):
            return batch_norm(y, **batch_norm_params)
    b = _s.variable("biases", (num_out,), initializer=("constant", float(bias)), trainable=trainable,
                    restore=restore)
    return as_tensor(y) + b.to(as_tensor(y).dtype)


@_s.add_arg_scope
def conv2d(inputs, num_filters_out, kernel_size, stride=1, padding="SAME", activation=torch.relu, stddev=0.01,
           bias=0.0, weight_decay=0, batch_norm_params=None, is_training=True, trainable=True, restore=True,
           scope=None, reuse=None):
    """ops.conv2d (inception/slim/ops.py:169-249): HWIO weights '<scope>/weights'."""
    x = as_tensor(inputs)
    kh, kw = _pair(kernel_size)
    with _s.variable_scope(scope, "Conv", reuse=reuse):
        reg = _s.l2_regularizer(weight_decay) if weight_decay and weight_decay > 0 else None
        w = _s.variable("weights", (num_filters_out, kh, kw, x.shape[-1]), initializer=("truncated_normal", stddev),
                        regularizer=reg, trainable=trainable, restore=restore, tf_layout="KRSC->HWIO")
        if batch_norm_params is None and activation in (torch.relu, E.relu, "relu"):
            b = _s.variable("biases", (num_filters_out,), initializer=("constant", float(bias)),
                            trainable=trainable, restore=restore)
            return F.conv2d(x, w, b, _pair(stride)[0], padding, relu=True)
        y = F.conv2d(x, w, None, _pair(stride)[0], padding)
        y = _bn_or_bias(y, num_filters_out, bias, batch_norm_params, is_training, trainable, restore)
    return _activate(y, activation)


@_s.add_arg_scope
def fc(inputs, num_units_out, activation=torch.relu, stddev=0.01, bias=0.0, weight_decay=0, batch_norm_params=None,
       is_training=True, trainable=True, restore=True, scope=None, reuse=None):
    """ops.fc (inception/slim/ops.py:252-320): weights [in, out]."""
    x = as_tensor(inputs)
    x = x.reshape(x.shape[0], -1)
    with _s.variable_scope(scope, "FC", reuse=reuse):
        reg = _s.l2_regularizer(weight_decay) if weight_decay and weight_decay > 0 else None
        w = _s.variable("weights", (x.shape[-1], num_units_out), initializer=("truncated_normal", stddev),
                        regularizer=reg, trainable=trainable, restore=restore)
        if batch_norm_params is None:
            b = _s.variable("biases", (num_units_out,), initializer=("constant", float(bias)), trainable=trainable,
                            restore=restore)
            relu = activation in (torch.relu, E.relu, "relu")
            y = F.linear(x, w, b, relu=relu)
            return y if relu else _activate(y, activation)
        y = F.linear(x, w, None)
        y = _bn_or_bias(y.reshape(y.shape[0], 1, 1, -1), num_units_out, bias, batch_norm_params, is_training,
                        trainable, restore).reshape(y.shape)
    return _activate(y, activation)


def one_hot_encoding(labels, num_classes, scope=None):
    """ops.one_hot_encoding: float32 [batch, num_classes]."""
    return torch.nn.functional.one_hot(labels.long().reshape(-1), num_classes).to(torch.float32)


@_s.add_arg_scope
def max_pool(inputs, kernel_size, stride=2, padding="VALID", scope=None):
    kh, kw = _pair(kernel_size)
    sh, sw = _pair(stride)
    return F.max_pool(as_tensor(inputs), (kh, kw), (sh, sw), padding)


@_s.add_arg_scope
def avg_pool(inputs, kernel_size, stride=2, padding="VALID", scope=None):
    kh, kw = _pair(kernel_size)
    sh, sw = _pair(stride)
    return F.avg_pool(as_tensor(inputs), (kh, kw), (sh, sw), padding)


@_s.add_arg_scope
def dropout(inputs, keep_prob=0.5, is_training=True, scope=None):
    if is_training and keep_prob < 1.0:
        return E.dropout(as_tensor(inputs), keep_prob)
    return inputs


def flatten(inputs, scope=None):
    x = as_tensor(inputs)
    if x.dim() < 2:
        raise ValueError("Inputs must have a least 2 dimensions")
    return x.reshape(x.shape[0], -1)


def repeat_op(repetitions, inputs, op, *args, **kwargs):
    """ops.repeat_op: ``op`` applied ``repetitions`` times under ``scope`` (default 'RepeatOp')."""
    scope = kwargs.pop("scope", None)
    with _s.variable_scope(scope, "RepeatOp"):
        tower = inputs
        for _ in range(repetitions):
            tower = op(tower, *args, **kwargs)
        return tower


# ---------------------------------------------------------------------------------------------
# losses.py (weight= keyword names of the old API)
def l1_regularizer(weight=1.0, scope=None):
    return _s.l1_regularizer(weight)


def l2_regularizer(weight=1.0, scope=None):
    return _s.l2_regularizer(weight)


def l1_l2_regularizer(weight_l1=1.0, weight_l2=1.0, scope=None):
    return _s.l1_l2_regularizer(weight_l1, weight_l2)


# ---------------------------------------------------------------------------------------------
# variables.py
def variable(name, shape=None, dtype=torch.float32, initializer=None, regularizer=None, trainable=True,
             collections=None, device="", restore=True):
    return _s.variable(name, shape, dtype, initializer, regularizer, trainable, collections,
                       device or None, restore)


def get_unique_variable(name):
    """The one variable named exactly ``name`` (variables.py:153-172)."""
    v = _s.get_store().vars.get(name)
    if v is None:
        raise ValueError("Couldn't find variable %s" % name)
    return v


def variable_device(device, name):
    """variables.variable_device: resolve a device fn / string for a variable."""
    return device(None) if callable(device) else device


ops = types.SimpleNamespace(
    batch_norm=batch_norm, conv2d=conv2d, fc=fc, one_hot_encoding=one_hot_encoding, max_pool=max_pool,
    avg_pool=avg_pool, dropout=dropout, flatten=flatten, repeat_op=repeat_op,
    UPDATE_OPS_COLLECTION=UPDATE_OPS_COLLECTION)
scopes = types.SimpleNamespace(arg_scope=_s.arg_scope, add_arg_scope=_s.add_arg_scope,
                               has_arg_scope=_s.has_arg_scope)
variables = types.SimpleNamespace(
    variable=variable, global_step=_s.global_step, get_variables=_s.get_variables,
    get_variables_to_restore=_s.get_variables_to_restore, get_variables_by_name=_s.get_variables_by_name,
    get_unique_variable=get_unique_variable, VariableDeviceChooser=_s.VariableDeviceChooser,
    variable_device=variable_device, MODEL_VARIABLES=MODEL_VARIABLES, VARIABLES_TO_RESTORE=VARIABLES_TO_RESTORE)
losses = types.SimpleNamespace(
    l1_regularizer=l1_regularizer, l2_regularizer=l2_regularizer, l1_l2_regularizer=l1_l2_regularizer,
    l1_loss=_s.losses.l1_loss, l2_loss=_s.losses.l2_loss, cross_entropy_loss=_s.losses.cross_entropy_loss,
    get_losses=_s.losses.get_losses, get_regularization_losses=_s.losses.get_regularization_losses,
    get_total_loss=_s.losses.get_total_loss, LOSSES_COLLECTION=LOSSES_COLLECTION)
