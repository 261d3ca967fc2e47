"""ResNet v1 (slim geometry): resnet_v1_{50,101,152,200}.

Structure and variable names follow reference vgg/nets/resnet_v1.py:78-375 and
vgg/nets/resnet_utils.py:59-272:
  * stride is applied in the 3x3 of the LAST unit of blocks 1-3 (spatial 56 -> 28 -> 14 -> 7 -> 7);
  * projection shortcut (1x1 conv + BN, no activation) only when the depth changes, otherwise
    ``subsample`` = 1x1 max-pool with the unit stride;
  * conv2d_same: explicit symmetric pad (k-1)//2 + VALID when stride > 1;
  * resnet_arg_scope: L2 1e-4, BN decay 0.997, eps 1e-5, scale=True, variance-scaling init,
    max_pool2d padding SAME.
Variables: resnet_v1_50/conv1/weights, resnet_v1_50/conv1/BatchNorm/{gamma,beta,moving_*},
resnet_v1_50/block1/unit_1/bottleneck_v1/{shortcut,conv1,conv2,conv3}/..., resnet_v1_50/logits/{weights,biases}.
"""

import torch

from ..ops import nn as F
from ..ops import fused
from ..ops.lazy import Subsampled, as_tensor
from .layers import Conv2d, Layer, _join, apply_activation, fused_enabled


def resnet_arg_scope(weight_decay=0.0001, batch_norm_decay=0.997, batch_norm_epsilon=1e-5, batch_norm_scale=True):
    return dict(weight_decay=weight_decay, init="variance_scaling",
                normalizer=dict(decay=batch_norm_decay, epsilon=batch_norm_epsilon, scale=batch_norm_scale,
                                bessel=True))


def subsample(x, factor, lazy=False):
    """1x1 max-pool with stride ``factor`` (resnet_utils.subsample).  ``lazy``: on the fused HIP path
    return a ``Subsampled`` view that the unit's output BN-apply reads strided (never stored)."""
    if factor == 1:
        return x
    if lazy and x.is_cuda and fused_enabled():
        return Subsampled(x, factor)
    return F.max_pool(as_tensor(x), 1, factor, "VALID")


def conv2d_same_padding(kernel, stride, rate=1):
    """resnet_utils.conv2d_same (reference vgg/nets/resnet_utils.py:77-122): stride 1 -> 'SAME';
    else explicit [pad_beg, pad_end] (pad_end = pad_beg + 1 for an even effective kernel) + VALID."""
    if stride == 1:
        return "SAME"
    keff = kernel + (kernel - 1) * (rate - 1)
    total = keff - 1
    beg = total // 2
    end = total - beg
    if end == beg:
        return (beg, beg)
    return ((beg, end), (beg, end))


class BottleneckV1(Layer):
    def __init__(self, scope, depth_in, depth, depth_bottleneck, stride, sc, rate=1):
        super().__init__(scope)
        self.stride = stride
        wd, init, bn = sc["weight_decay"], sc["init"], sc["normalizer"]
        if depth != depth_in:
            self.shortcut = Conv2d(_join(scope, "shortcut"), depth_in, depth, 1, stride, "SAME", activation=None,
                                   normalizer=bn, weight_decay=wd, init=init)
        else:
            self.shortcut = None
        self.conv1 = Conv2d(_join(scope, "conv1"), depth_in, depth_bottleneck, 1, 1, "SAME", "relu", bn, None, wd, init)
        self.conv2 = Conv2d(_join(scope, "conv2"), depth_bottleneck, depth_bottleneck, 3, stride,
                            conv2d_same_padding(3, stride, rate), "relu", bn, None, wd, init, rate=rate)
        self.conv3 = Conv2d(_join(scope, "conv3"), depth_bottleneck, depth, 1, 1, "SAME", None, bn, None, wd, init)

    def forward(self, x, training=True, end_points=None):
        if self.shortcut is not None:
            # projection shortcut and conv1: sibling 1x1 conv+BNs of x with one merged backward (ops.fused).  (A merged
            # FORWARD, as Inception's heads have, was measured +0.31..+0.41 % step here - the 512 + 128 -> 640-channel
            # conv loses the 8-wave tile the 512-channel shortcut gets alone, profiles/ab/r4_ab_fwd_dtile_resnet.log,
            # r4_ab_rfwd_resnet.log - and was removed.)
            with fused.sibling_group(x, training and end_points is None):
                sc = self.shortcut(x, training)
                r1 = self.conv1(x, training)
        else:
            sc = subsample(x, self.stride, lazy=self.conv3.bn is not None and end_points is None)
            r1 = self.conv1(x, training)
        r2 = self.conv2(r1, training)
        if end_points is not None:
            # slim collects every conv output (outputs_collections) plus the unit output
            r3 = self.conv3(r2, training)
            y = apply_activation(as_tensor(r3) + as_tensor(sc), "relu")
            if self.shortcut is not None:
                end_points[self.shortcut.scope] = as_tensor(sc)
            for c, v in ((self.conv1, r1), (self.conv2, r2), (self.conv3, r3)):
                end_points[c.scope] = as_tensor(v)
            end_points[self.scope] = y
            return y
        return self.conv3(r2, training, residual=sc, residual_act="relu")


def stack_blocks_plan(blocks, output_stride=None, store_non_strided_activations=False):
    """The unit schedule of resnet_utils.stack_blocks_dense (reference vgg/nets/resnet_utils.py:125-219).

    blocks: [(base_depth, num_units, stride)], stride applied in the LAST unit of the block
    (resnet_v1_block / resnet_v2_block).  Returns [([(unit_stride, unit_rate), ...], block_end_subsample)]:
    once the running stride reaches ``output_stride`` every further unit runs with stride 1 and an
    atrous rate that absorbs the skipped strides.  ``store_non_strided_activations`` moves the last
    unit's stride to a subsample at the block end (the block endpoint is then undecimated)."""
    current_stride, rate = 1, 1
    plan = []
    for base, n, stride in blocks:
        units, block_stride = [], 1
        for i in range(n):
            s = stride if i == n - 1 else 1
            if store_non_strided_activations and i == n - 1:
                block_stride, s = s, 1
            if output_stride is not None and current_stride == output_stride:
                units.append((1, rate))
                rate *= s
            else:
                units.append((s, 1))
                current_stride *= s
                if output_stride is not None and current_stride > output_stride:
                    raise ValueError("The target output_stride cannot be reached.")
        if output_stride is not None and current_stride == output_stride:
            rate *= block_stride
            sub = 1
        else:
            sub = block_stride
            current_stride *= block_stride
            if output_stride is not None and current_stride > output_stride:
                raise ValueError("The target output_stride cannot be reached.")
        plan.append((units, sub))
    if output_stride is not None and current_stride != output_stride:
        raise ValueError("The target output_stride cannot be reached.")
    return plan


def resnet_v1_block(scope, base_depth, num_units, stride):
    """resnet_v1.resnet_v1_block: (base_depth, num_units, stride) in this module's block format."""
    return (base_depth, num_units, stride)


BLOCKS = {
    50: [(64, 3, 2), (128, 4, 2), (256, 6, 2), (512, 3, 1)],
    101: [(64, 3, 2), (128, 4, 2), (256, 23, 2), (512, 3, 1)],
    152: [(64, 3, 2), (128, 8, 2), (256, 36, 2), (512, 3, 1)],
    200: [(64, 3, 2), (128, 24, 2), (256, 36, 2), (512, 3, 1)],
}


class ResNetV1(Layer):
    default_image_size = 224

    def __init__(self, depth=50, num_classes=1000, global_pool=True, spatial_squeeze=True, scope=None,
                 arg_scope=None, blocks=None, include_root_block=True, in_channels=3, output_stride=None,
                 store_non_strided_activations=False):
        scope = scope or "resnet_v1_%d" % depth
        super().__init__(scope)
        sc = arg_scope or resnet_arg_scope()
        self.num_classes, self.global_pool, self.spatial_squeeze = num_classes, global_pool, spatial_squeeze
        self.include_root_block = include_root_block
        self.output_stride = output_stride
        cin = in_channels
        if include_root_block:
            if output_stride is not None:
                if output_stride % 4 != 0:
                    raise ValueError("The output_stride needs to be a multiple of 4.")
                output_stride //= 4
            self.conv1 = Conv2d(_join(scope, "conv1"), cin, 64, 7, 2, conv2d_same_padding(7, 2), "relu",
                                sc["normalizer"], None, sc["weight_decay"], sc["init"])
            cin = 64
        blocks = blocks or BLOCKS[depth]
        plan = stack_blocks_plan(blocks, output_stride, store_non_strided_activations)
        units = []
        self.block_ends = []
        for bi, ((base, n, _), (uplan, sub)) in enumerate(zip(blocks, plan)):
            for ui, (s, rate) in enumerate(uplan):
                units.append(BottleneckV1(_join(scope, "block%d/unit_%d/bottleneck_v1" % (bi + 1, ui + 1)), cin,
                                          base * 4, base, s, sc, rate=rate))
                cin = base * 4
            self.block_ends.append((len(units) - 1, _join(scope, "block%d" % (bi + 1)), sub))
        self.units = torch.nn.ModuleList(units)
        self.num_features = cin
        if num_classes:
            self.logits = Conv2d(_join(scope, "logits"), cin, num_classes, 1, 1, "SAME", None, None, True,
                                 sc["weight_decay"], sc["init"])
        else:
            self.logits = None

    def forward(self, x, training=True, end_points=None):
        net = x
        if self.include_root_block:
            net = self.conv1(net, training)
            if end_points is not None:
                end_points[self.conv1.scope] = as_tensor(net)
            net = F.max_pool(net, 3, 2, "SAME")
        ends = {i: (name, sub) for i, name, sub in self.block_ends}
        for i, u in enumerate(self.units):
            net = u(net, training, end_points) if end_points is not None else u(net, training)
            if i in ends:
                name, sub = ends[i]
                if end_points is not None:
                    end_points[name] = net
                net = subsample(net, sub)
        if self.global_pool:
            # (bf16 when the logits layer follows: it computes in bf16, the cast launch disappears)
            net = F.global_avg_pool(net, out_bf16=self.logits is not None).reshape(net.shape[0], 1, 1, -1)
            if end_points is not None:
                end_points["global_pool"] = net
        if self.logits is not None:
            net = self.logits(net.to(torch.bfloat16) if net.is_cuda else net, training)
            if end_points is not None:
                end_points[self.scope + "/logits"] = net
            if self.spatial_squeeze:
                if net.shape[1] != 1 or net.shape[2] != 1:
                    raise ValueError("spatial_squeeze needs a 1x1 logits map, got %s" % (tuple(net.shape),))
                net = net.reshape(net.shape[0], -1)
                if end_points is not None:
                    end_points[self.scope + "/spatial_squeeze"] = net
            if end_points is not None:
                end_points["predictions"] = torch.softmax(net.float(), -1)
        return net


def resnet_v1_50(num_classes=1000, **kw):
    return ResNetV1(50, num_classes, **kw)


def resnet_v1_101(num_classes=1000, **kw):
    return ResNetV1(101, num_classes, **kw)


def resnet_v1_152(num_classes=1000, **kw):
    return ResNetV1(152, num_classes, **kw)


def resnet_v1_200(num_classes=1000, **kw):
    return ResNetV1(200, num_classes, **kw)
