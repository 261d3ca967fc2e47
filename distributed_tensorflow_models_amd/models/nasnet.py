"""NASNet-A (CIFAR / Mobile / Large) and PNASNet-5 Large on the functional slim facade.

Cell programs, hidden-state wiring, stems, aux heads and hyper-parameters follow the reference
(vgg/nets/nasnet/nasnet_utils.py:43-497, nasnet.py:37-526, pnasnet.py:30-197); endpoint shapes
are golden-tested in tests/test_models.py.  Separable convs run on the HIP depthwise kernels +
the implicit-GEMM pointwise conv; NHWC only (the reference's NCHW switch is a CUDA-layout
concern that does not apply here).

drop_path follows the reference "v3" schedule: keep = 1 - (cell+1)/total_cells * min(1, step /
total_training_steps) * (1 - drop_path_keep_prob); the training step comes from
``set_training_step`` (the trainer's global step), 0 by default (=> no drop, as in TF at step 0).
"""
import copy

import torch

from ..compat import slim
from ..ops import nn as F
from ..ops.lazy import as_tensor

_STEP = [0]


def set_training_step(step):
    _STEP[0] = int(step)


class HParams(dict):
    __getattr__ = dict.__getitem__

    def __setattr__(self, k, v):
        self[k] = v


def cifar_config():
    return HParams(stem_multiplier=3.0, drop_path_keep_prob=0.6, num_cells=18, use_aux_head=1, num_conv_filters=32,
                   dense_dropout_keep_prob=1.0, filter_scaling_rate=2.0, num_reduction_layers=2,
                   skip_reduction_layer_input=0, total_training_steps=937500)


def large_imagenet_config():
    return HParams(stem_multiplier=3.0, dense_dropout_keep_prob=0.5, num_cells=18, filter_scaling_rate=2.0,
                   num_conv_filters=168, drop_path_keep_prob=0.7, use_aux_head=1, num_reduction_layers=2,
                   skip_reduction_layer_input=1, total_training_steps=250000)


def mobile_imagenet_config():
    return HParams(stem_multiplier=1.0, dense_dropout_keep_prob=0.5, num_cells=12, filter_scaling_rate=2.0,
                   drop_path_keep_prob=1.0, num_conv_filters=44, use_aux_head=1, num_reduction_layers=2,
                   skip_reduction_layer_input=0, total_training_steps=250000)


def pnasnet_large_config():
    return HParams(stem_multiplier=3.0, dense_dropout_keep_prob=0.5, num_cells=12, filter_scaling_rate=2.0,
                   num_conv_filters=216, drop_path_keep_prob=0.6, use_aux_head=1, num_reduction_layers=2,
                   skip_reduction_layer_input=1, total_training_steps=250000)


# ---------------------------------------------------------------------------------------------
# utilities (nasnet_utils)
def calc_reduction_layers(num_cells, num_reduction_layers):
    return [int(float(i) / (num_reduction_layers + 1) * num_cells) for i in range(1, num_reduction_layers + 1)]


def _relu(x):
    return torch.relu(as_tensor(x))


def global_avg_pool(x):
    return F.global_avg_pool(x)


def factorized_reduction(net, output_filters, stride):
    """Stride-2 reduction as two half-width 1x1 convs on the input and on its one-pixel shift."""
    assert output_filters % 2 == 0
    if stride == 1:
        net = slim.conv2d(net, output_filters, 1, scope="path_conv")
        return slim.batch_norm(net, scope="path_bn")
    x = as_tensor(net)
    p1 = slim.conv2d(x[:, ::stride, ::stride, :], output_filters // 2, 1, scope="path1_conv")
    shifted = torch.nn.functional.pad(x[:, 1:, 1:, :], (0, 0, 0, 1, 0, 1))
    p2 = slim.conv2d(shifted[:, ::stride, ::stride, :], output_filters // 2, 1, scope="path2_conv")
    return slim.batch_norm(torch.cat([as_tensor(p1), as_tensor(p2)], -1), scope="final_path_bn")


def drop_path(net, keep_prob, is_training=True):
    x = as_tensor(net)
    if not is_training or keep_prob >= 1.0:
        return x
    mask = torch.floor(keep_prob + torch.rand(x.shape[0], 1, 1, 1, device=x.device))
    return x / keep_prob * mask.to(x.dtype)


def _op_info(op):
    parts = op.split("_")
    k = int(parts[1].split("x")[0]) if "x" in parts[1] else int(parts[-1].split("x")[0])
    layers = 1 if "x" in parts[-1] else int(parts[-1])
    return layers, k


def _stacked_separable_conv(net, stride, op, filters):
    layers, k = _op_info(op)
    for i in range(layers):
        net = _relu(net)
        net = slim.separable_conv2d(net, filters, k, depth_multiplier=1, stride=stride,
                                    scope="separable_{0}x{0}_{1}".format(k, i + 1))
        net = slim.batch_norm(net, scope="bn_sep_{0}x{0}_{1}".format(k, i + 1))
        stride = 1
    return net


def _pooling(net, stride, op):
    kind = op.split("_")[0]
    k = int(op.split("_")[-1].split("x")[0])
    if kind == "avg":
        return slim.avg_pool2d(net, k, stride=stride, padding="SAME")
    if kind == "max":
        return slim.max_pool2d(net, k, stride=stride, padding="SAME")
    raise NotImplementedError(op)


class BaseCell:
    """Five pairwise combinations of hidden states (nasnet_utils.NasNetABaseCell)."""
    operations = used_hiddenstates = hiddenstate_indices = None

    def __init__(self, num_conv_filters, drop_path_keep_prob, total_num_cells, total_training_steps):
        self.num_conv_filters = num_conv_filters
        self.drop_path_keep_prob = drop_path_keep_prob
        self.total_num_cells = total_num_cells
        self.total_training_steps = total_training_steps
        self.is_training = True

    def _reduce_prev_layer(self, prev, curr):
        if prev is None:
            return curr
        prev, curr = as_tensor(prev), as_tensor(curr)
        if curr.shape[2] != prev.shape[2]:
            return factorized_reduction(_relu(prev), self.filter_size, 2)
        if self.filter_size != prev.shape[-1]:
            p = slim.conv2d(_relu(prev), self.filter_size, 1, scope="prev_1x1")
            return slim.batch_norm(p, scope="prev_bn")
        return prev

    def __call__(self, net, scope, filter_scaling=1, stride=1, prev_layer=None, cell_num=-1):
        self.cell_num = cell_num
        self.filter_size = int(self.num_conv_filters * filter_scaling)
        with slim.variable_scope(scope):
            prev = self._reduce_prev_layer(prev_layer, net)
            h = slim.batch_norm(slim.conv2d(_relu(net), self.filter_size, 1, scope="1x1"), scope="beginning_bn")
            states = [as_tensor(h), as_tensor(prev)]
            for it in range(5):
                with slim.variable_scope("comb_iter_%d" % it):
                    li, ri = self.hiddenstate_indices[2 * it], self.hiddenstate_indices[2 * it + 1]
                    with slim.variable_scope("left"):
                        h1 = self._apply(states[li], self.operations[2 * it], stride, li < 2)
                    with slim.variable_scope("right"):
                        h2 = self._apply(states[ri], self.operations[2 * it + 1], stride, ri < 2)
                    states.append(as_tensor(h1) + as_tensor(h2))
            with slim.variable_scope("cell_output"):
                return self._combine_unused(states)

    def _apply(self, net, op, stride, from_original):
        if stride > 1 and not from_original:
            stride = 1
        cin = as_tensor(net).shape[-1]
        if "separable" in op:
            net = _stacked_separable_conv(net, stride, op, self.filter_size)
        elif op == "none":
            if stride > 1 or cin != self.filter_size:
                net = slim.conv2d(_relu(net), self.filter_size, 1, stride=stride, scope="1x1")
                net = slim.batch_norm(net, scope="bn_1")
        elif "pool" in op:
            net = _pooling(net, stride, op)
            if cin != self.filter_size:
                net = slim.batch_norm(slim.conv2d(net, self.filter_size, 1, stride=1, scope="1x1"), scope="bn_1")
        else:
            raise ValueError("Unimplemented operation", op)
        if op != "none":
            net = self._drop_path(net)
        return net

    def _combine_unused(self, states):
        final_h, final_c = states[-1].shape[2], states[-1].shape[-1]
        for idx, used in enumerate(self.used_hiddenstates):
            h, c = states[idx].shape[2], states[idx].shape[-1]
            if (final_c != c or final_h != h) and not used:
                with slim.variable_scope("reduction_%d" % idx):
                    states[idx] = as_tensor(factorized_reduction(states[idx], final_c, 2 if final_h != h else 1))
        return torch.cat([s for s, used in zip(states, self.used_hiddenstates) if not used], -1)

    def _drop_path(self, net):
        keep = self.drop_path_keep_prob
        if keep >= 1.0 or not self.is_training:
            return net
        layer_ratio = (self.cell_num + 1) / float(self.total_num_cells)
        keep = 1 - layer_ratio * (1 - keep)
        ratio = min(1.0, _STEP[0] / float(self.total_training_steps))
        keep = 1 - ratio * (1 - keep)
        return drop_path(net, keep, True)


class NasNetANormalCell(BaseCell):
    operations = ["separable_5x5_2", "separable_3x3_2", "separable_5x5_2", "separable_3x3_2", "avg_pool_3x3",
                  "none", "avg_pool_3x3", "avg_pool_3x3", "separable_3x3_2", "none"]
    used_hiddenstates = [1, 0, 0, 0, 0, 0, 0]
    hiddenstate_indices = [0, 1, 1, 1, 0, 1, 1, 1, 0, 0]


class NasNetAReductionCell(BaseCell):
    operations = ["separable_5x5_2", "separable_7x7_2", "max_pool_3x3", "separable_7x7_2", "avg_pool_3x3",
                  "separable_5x5_2", "none", "avg_pool_3x3", "separable_3x3_2", "max_pool_3x3"]
    used_hiddenstates = [1, 1, 1, 0, 0, 0, 0]
    hiddenstate_indices = [0, 1, 0, 1, 0, 1, 3, 2, 2, 0]


class PNasNetNormalCell(BaseCell):
    operations = ["separable_5x5_2", "max_pool_3x3", "separable_7x7_2", "max_pool_3x3", "separable_5x5_2",
                  "separable_3x3_2", "separable_3x3_2", "max_pool_3x3", "separable_3x3_2", "none"]
    used_hiddenstates = [1, 1, 0, 0, 0, 0, 0]
    hiddenstate_indices = [1, 1, 0, 0, 0, 0, 4, 0, 1, 0]


# ---------------------------------------------------------------------------------------------
# arg scopes, stems, heads (nasnet.py)
class _ArgScopes:
    def __init__(self, weight_decay, bn_decay, bn_eps):
        self.ctx = [
            slim.arg_scope([slim.fully_connected, slim.conv2d, slim.separable_conv2d],
                           weights_regularizer=slim.l2_regularizer(weight_decay),
                           weights_initializer=slim.variance_scaling_initializer(mode="FAN_OUT")),
            slim.arg_scope([slim.fully_connected], activation_fn=None, scope="FC"),
            slim.arg_scope([slim.conv2d, slim.separable_conv2d], activation_fn=None, biases_initializer=None),
            slim.arg_scope([slim.batch_norm], decay=bn_decay, epsilon=bn_eps, scale=True),
        ]

    def __enter__(self):
        for c in self.ctx:
            c.__enter__()

    def __exit__(self, *a):
        for c in reversed(self.ctx):
            c.__exit__(*a)


ARG_SCOPES = {"cifar": (5e-4, 0.9, 1e-5), "mobile": (4e-5, 0.9997, 1e-3), "large": (5e-5, 0.9997, 1e-3),
              "pnasnet": (4e-5, 0.9997, 1e-3)}


def _build_aux_head(net, ep, num_classes, scope):
    with slim.variable_scope(scope):
        with slim.variable_scope("aux_logits"):
            a = slim.avg_pool2d(net, 5, stride=3, padding="VALID")
            a = _relu(slim.batch_norm(slim.conv2d(a, 128, 1, scope="proj"), scope="aux_bn0"))
            a = slim.conv2d(a, 768, (a.shape[1], a.shape[2]), padding="VALID")
            a = _relu(slim.batch_norm(a, scope="aux_bn1"))
            ep["AuxLogits"] = slim.fully_connected(slim.flatten(a), num_classes)


def _imagenet_stem(images, hp, stem_cell):
    net = slim.conv2d(images, int(32 * hp.stem_multiplier), 3, stride=2, padding="VALID", scope="conv0")
    net = as_tensor(slim.batch_norm(net, scope="conv0_bn"))
    outs = [None, net]
    fs = 1.0 / (hp.filter_scaling_rate ** 2)
    for i in range(2):
        net = stem_cell(net, scope="cell_stem_%d" % i, filter_scaling=fs, stride=2, prev_layer=outs[-2], cell_num=i)
        outs.append(net)
        fs *= hp.filter_scaling_rate
    return net, outs


def _cifar_stem(images, hp):
    net = slim.conv2d(images, int(hp.num_conv_filters * hp.stem_multiplier), 3, scope="l1_stem_3x3")
    net = as_tensor(slim.batch_norm(net, scope="l1_stem_bn"))
    return net, [None, net]


def _final_layer(net, ep, num_classes, hp, final_endpoint):
    with slim.variable_scope("final_layer"):
        net = ep["global_pool"] = global_avg_pool(_relu(net))
        if final_endpoint == "global_pool" or not num_classes:
            return net, True
        net = slim.dropout(net, hp.dense_dropout_keep_prob, scope="dropout")
        logits = ep["Logits"] = slim.fully_connected(net, num_classes)
        ep["Predictions"] = torch.softmax(as_tensor(logits).float(), -1)
        return logits, final_endpoint in ("Logits", "Predictions")


def _build_nasnet_base(images, normal_cell, reduction_cell, num_classes, hp, is_training, stem_type,
                       final_endpoint=None):
    ep = {}
    red = calc_reduction_layers(hp.num_cells, hp.num_reduction_layers)
    if stem_type == "imagenet":
        net, outs = _imagenet_stem(images, hp, reduction_cell)
    else:
        net, outs = _cifar_stem(images, hp)
    ep["Stem"] = net
    if final_endpoint == "Stem":
        return net, ep
    aux_idx = [red[1] - 1] if len(red) >= 2 else []
    fs = 1.0
    true_cell = 2 if stem_type == "imagenet" else 0
    prev = None
    for c in range(hp.num_cells):
        if hp.skip_reduction_layer_input:
            prev = outs[-2]
        if c in red:
            fs *= hp.filter_scaling_rate
            name = "Reduction_Cell_%d" % red.index(c)
            net = ep[name] = reduction_cell(net, scope="reduction_cell_%d" % red.index(c), filter_scaling=fs,
                                            stride=2, prev_layer=outs[-2], cell_num=true_cell)
            if final_endpoint == name:
                return net, ep
            true_cell += 1
            outs.append(net)
        if not hp.skip_reduction_layer_input:
            prev = outs[-2]
        net = ep["Cell_%d" % c] = normal_cell(net, scope="cell_%d" % c, filter_scaling=fs, stride=1,
                                              prev_layer=prev, cell_num=true_cell)
        if final_endpoint == "Cell_%d" % c:
            return net, ep
        true_cell += 1
        if hp.use_aux_head and c in aux_idx and num_classes and is_training:
            _build_aux_head(_relu(net), ep, num_classes, scope="aux_%d" % c)
        outs.append(net)
    out, stop = _final_layer(net, ep, num_classes, hp, final_endpoint)
    return out, ep


def _nasnet(images, num_classes, is_training, config, default_cfg, scopes, stem, extra_cells, final_endpoint):
    hp = copy.deepcopy(config) if config is not None else default_cfg()
    if not is_training:
        hp.drop_path_keep_prob = 1.0
    total = hp.num_cells + 2 + extra_cells
    normal = NasNetANormalCell(hp.num_conv_filters, hp.drop_path_keep_prob, total, hp.total_training_steps)
    reduction = NasNetAReductionCell(hp.num_conv_filters, hp.drop_path_keep_prob, total, hp.total_training_steps)
    normal.is_training = reduction.is_training = is_training
    with _ArgScopes(*ARG_SCOPES[scopes]), slim.arg_scope([slim.dropout, slim.batch_norm], is_training=is_training):
        logits, ep = _build_nasnet_base(images, normal, reduction, num_classes, hp, is_training, stem, final_endpoint)
    if is_training and "AuxLogits" in ep and final_endpoint is None:
        return (logits, ep["AuxLogits"]), ep
    return logits, ep


def build_nasnet_cifar(images, num_classes=10, is_training=True, config=None, final_endpoint=None):
    return _nasnet(images, num_classes, is_training, config, cifar_config, "cifar", "cifar", 0, final_endpoint)


def build_nasnet_mobile(images, num_classes=1001, is_training=True, final_endpoint=None, config=None):
    return _nasnet(images, num_classes, is_training, config, mobile_imagenet_config, "mobile", "imagenet", 2,
                   final_endpoint)


def build_nasnet_large(images, num_classes=1001, is_training=True, final_endpoint=None, config=None):
    return _nasnet(images, num_classes, is_training, config, large_imagenet_config, "large", "imagenet", 2,
                   final_endpoint)


def build_pnasnet_large(images, num_classes=1001, is_training=True, final_endpoint=None, config=None):
    hp = copy.deepcopy(config) if config is not None else pnasnet_large_config()
    if not is_training:
        hp.drop_path_keep_prob = 1.0
    cell = PNasNetNormalCell(hp.num_conv_filters, hp.drop_path_keep_prob, hp.num_cells + 2, hp.total_training_steps)
    cell.is_training = is_training
    ep = {}
    with _ArgScopes(*ARG_SCOPES["pnasnet"]), slim.arg_scope([slim.dropout, slim.batch_norm], is_training=is_training):
        red = calc_reduction_layers(hp.num_cells, hp.num_reduction_layers)
        net, outs = _imagenet_stem(images, hp, cell)
        ep["Stem"] = net
        if final_endpoint == "Stem":
            return net, ep
        aux_idx = [red[1] - 1] if len(red) >= 2 else []
        fs = 1.0
        true_cell = 2
        for c in range(hp.num_cells):
            is_red = c in red
            if is_red:
                fs *= hp.filter_scaling_rate
            net = ep["Cell_%d" % c] = cell(net, scope="cell_%d" % c, filter_scaling=fs, stride=2 if is_red else 1,
                                           prev_layer=outs[-2], cell_num=true_cell)
            if final_endpoint == "Cell_%d" % c:
                return net, ep
            true_cell += 1
            outs.append(net)
            if hp.use_aux_head and c in aux_idx and num_classes and is_training:
                _build_aux_head(_relu(net), ep, num_classes, scope="aux_%d" % c)
        logits, _stop = _final_layer(net, ep, num_classes, hp, final_endpoint)
    if is_training and "AuxLogits" in ep and final_endpoint is None:
        return (logits, ep["AuxLogits"]), ep
    return logits, ep


build_nasnet_cifar.default_image_size = 32
build_nasnet_mobile.default_image_size = 224
build_nasnet_large.default_image_size = 331
build_pnasnet_large.default_image_size = 331
