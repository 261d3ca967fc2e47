"""TF-Slim model zoo written against the functional slim facade (compat.slim) - the nets_factory
registry of the reference (vgg/nets/nets_factory.py:39-100).  Structures, endpoint names and
variable names follow the slim definitions (reference vgg/nets/*.py); each model is verified
against the reference tests' golden numbers (tests/test_models.py).

Contents: resnet_v2_{50,101,152,200} (slim pre-activation), inception_v1, inception_v2,
inception_v3 (new slim; ``cifar_variant`` = the reference's VALID->SAME patch), inception_v4,
inception_resnet_v2, mobilenet_v1 (+0.75/0.5/0.25), mobilenet_v2.
"""
import torch

from ..compat import slim
from ..ops import nn as F
from ..ops.lazy import as_tensor

relu = torch.relu


def _relu6(x):
    from ..ops.activation import relu6
    return relu6(as_tensor(x))


def _cat(ts):
    return torch.cat([as_tensor(t) for t in ts], dim=-1)


def _squeeze(net):
    net = as_tensor(net)
    if net.shape[1] != 1 or net.shape[2] != 1:
        raise ValueError("spatial dims %s cannot be squeezed" % (tuple(net.shape),))
    return net.reshape(net.shape[0], -1)


def _bn_params(decay=0.9997, eps=0.001, scale=False):
    return dict(decay=decay, epsilon=eps, scale=scale)


# =============================================================================================
# ResNet v2 (slim): vgg/nets/resnet_v2.py:61-337 -- preact bottleneck, postnorm, logits 1x1
def _subsample(x, factor, scope=None):
    return x if factor == 1 else F.max_pool(x, 1, factor, "VALID")


def _conv2d_same(x, num_outputs, k, stride, scope, rate=1):
    """resnet_utils.conv2d_same: SAME for stride 1, else explicit symmetric pad of the (dilated)
    kernel + VALID (reference vgg/nets/resnet_utils.py:77-122)."""
    if stride == 1:
        return slim.conv2d(x, num_outputs, k, stride=1, rate=rate, padding="SAME", scope=scope)
    pad = ((k - 1) * rate) // 2
    return slim.conv2d(x, num_outputs, k, stride=stride, rate=rate, padding=(pad, pad), scope=scope)


def _bottleneck_v2(x, depth, depth_bottleneck, stride, scope, rate=1, ep=None):
    with slim.variable_scope(scope):
        with slim.variable_scope("bottleneck_v2") as vs:
            depth_in = as_tensor(x).shape[-1]
            preact = slim.batch_norm(x, activation_fn=relu, scope="preact")
            if depth == depth_in:
                shortcut = _subsample(x, stride)
            else:
                shortcut = slim.conv2d(preact, depth, 1, stride=stride, normalizer_fn=None, activation_fn=None,
                                       scope="shortcut")
                if ep is not None:
                    ep[vs + "/shortcut"] = shortcut
            r = slim.conv2d(preact, depth_bottleneck, 1, stride=1, scope="conv1")
            r2 = _conv2d_same(r, depth_bottleneck, 3, stride, "conv2", rate=rate)
            r3 = slim.conv2d(r2, depth, 1, stride=1, normalizer_fn=None, activation_fn=None, scope="conv3")
            out = as_tensor(shortcut) + as_tensor(r3)
            if ep is not None:
                for name, v in (("conv1", r), ("conv2", r2), ("conv3", r3)):
                    ep[vs + "/" + name] = v
                ep[vs] = out
            return out


RESNET_V2_BLOCKS = {50: [3, 4, 6, 3], 101: [3, 4, 23, 3], 152: [3, 8, 36, 3], 200: [3, 24, 36, 3]}


def resnet_v2_block(scope, base_depth, num_units, stride):
    """resnet_v2.resnet_v2_block (stride in the last unit) as (base_depth, num_units, stride)."""
    return (base_depth, num_units, stride)


def resnet_v2(images, num_classes=1000, is_training=True, depth=50, weight_decay=0.0001, scope=None,
              global_pool=True, spatial_squeeze=True, blocks=None, output_stride=None, include_root_block=True,
              store_non_strided_activations=False):
    """slim resnet_v2 generator (reference vgg/nets/resnet_v2.py:111-224): pre-activation
    bottlenecks, root conv without BN, ``postnorm`` BN-ReLU, atrous ``output_stride``.  Endpoints:
    every conv output, unit, block, global_pool, logits, spatial_squeeze, predictions."""
    from .resnet_v1 import stack_blocks_plan
    scope = scope or "resnet_v2_%d" % depth
    ep = {}
    bn = dict(decay=0.997, epsilon=1e-5, scale=True)
    if blocks is None:
        blocks = [(base, n, 2 if bi < 3 else 1) for bi, (base, n) in
                  enumerate(zip([64, 128, 256, 512], RESNET_V2_BLOCKS[depth]))]
    if include_root_block and output_stride is not None:
        if output_stride % 4 != 0:
            raise ValueError("The output_stride needs to be a multiple of 4.")
        output_stride //= 4
    plan = stack_blocks_plan(blocks, output_stride, store_non_strided_activations)
    with slim.arg_scope([slim.conv2d], weights_regularizer=slim.l2_regularizer(weight_decay),
                        weights_initializer=slim.variance_scaling_initializer(), activation_fn=relu,
                        normalizer_fn=slim.batch_norm, normalizer_params=bn):
        with slim.arg_scope([slim.batch_norm], **bn), slim.arg_scope([slim.max_pool2d], padding="SAME"):
            with slim.variable_scope(scope) as vs:
                net = images
                if include_root_block:
                    with slim.arg_scope([slim.conv2d], activation_fn=None, normalizer_fn=None):
                        net = _conv2d_same(net, 64, 7, 2, "conv1")
                    ep[vs + "/conv1"] = net
                    net = slim.max_pool2d(net, 3, stride=2, scope="pool1")
                for bi, ((base, n, _), (uplan, sub)) in enumerate(zip(blocks, plan)):
                    with slim.variable_scope("block%d" % (bi + 1)):
                        for u, (stride, rate) in enumerate(uplan):
                            net = _bottleneck_v2(net, base * 4, base, stride, "unit_%d" % (u + 1), rate, ep)
                    ep["%s/block%d" % (vs, bi + 1)] = net
                    net = _subsample(net, sub)
                net = slim.batch_norm(net, activation_fn=relu, scope="postnorm")
                if global_pool:
                    net = F.global_avg_pool(net).reshape(net.shape[0], 1, 1, -1)
                    ep["global_pool"] = net
                if num_classes:
                    net = slim.conv2d(net, num_classes, 1, activation_fn=None, normalizer_fn=None, scope="logits")
                    ep[vs + "/logits"] = net
                    if spatial_squeeze:
                        net = _squeeze(net)
                        ep[vs + "/spatial_squeeze"] = net
                    ep["predictions"] = torch.softmax(as_tensor(net).float(), -1)
    return net, ep


# =============================================================================================
# Inception v1 (vgg/nets/inception_v1.py:29-327)
def _mixed_v1(net, name, b0, b1a, b1b, b2a, b2b, b3, conv5_name="Conv2d_0b_3x3"):
    with slim.variable_scope(name):
        with slim.variable_scope("Branch_0"):
            x0 = slim.conv2d(net, b0, 1, scope="Conv2d_0a_1x1")
        with slim.variable_scope("Branch_1"):
            x1 = slim.conv2d(net, b1a, 1, scope="Conv2d_0a_1x1")
            x1 = slim.conv2d(x1, b1b, 3, scope="Conv2d_0b_3x3")
        with slim.variable_scope("Branch_2"):
            x2 = slim.conv2d(net, b2a, 1, scope="Conv2d_0a_1x1")
            x2 = slim.conv2d(x2, b2b, 3, scope=conv5_name)
        with slim.variable_scope("Branch_3"):
            x3 = slim.max_pool2d(net, 3, stride=1, scope="MaxPool_0a_3x3")
            x3 = slim.conv2d(x3, b3, 1, scope="Conv2d_0b_1x1")
        return _cat([x0, x1, x2, x3])


def inception_v1_base(images, ep):
    with slim.arg_scope([slim.conv2d, slim.fully_connected], weights_initializer=slim.trunc_normal(stddev=0.01)):
        with slim.arg_scope([slim.conv2d, slim.max_pool2d], stride=1, padding="SAME"):
            net = ep["Conv2d_1a_7x7"] = slim.conv2d(images, 64, 7, stride=2, scope="Conv2d_1a_7x7")
            net = ep["MaxPool_2a_3x3"] = slim.max_pool2d(net, 3, stride=2, scope="MaxPool_2a_3x3")
            net = ep["Conv2d_2b_1x1"] = slim.conv2d(net, 64, 1, scope="Conv2d_2b_1x1")
            net = ep["Conv2d_2c_3x3"] = slim.conv2d(net, 192, 3, scope="Conv2d_2c_3x3")
            net = ep["MaxPool_3a_3x3"] = slim.max_pool2d(net, 3, stride=2, scope="MaxPool_3a_3x3")
            net = ep["Mixed_3b"] = _mixed_v1(net, "Mixed_3b", 64, 96, 128, 16, 32, 32)
            net = ep["Mixed_3c"] = _mixed_v1(net, "Mixed_3c", 128, 128, 192, 32, 96, 64)
            net = ep["MaxPool_4a_3x3"] = slim.max_pool2d(net, 3, stride=2, scope="MaxPool_4a_3x3")
            net = ep["Mixed_4b"] = _mixed_v1(net, "Mixed_4b", 192, 96, 208, 16, 48, 64)
            net = ep["Mixed_4c"] = _mixed_v1(net, "Mixed_4c", 160, 112, 224, 24, 64, 64)
            net = ep["Mixed_4d"] = _mixed_v1(net, "Mixed_4d", 128, 128, 256, 24, 64, 64)
            net = ep["Mixed_4e"] = _mixed_v1(net, "Mixed_4e", 112, 144, 288, 32, 64, 64)
            net = ep["Mixed_4f"] = _mixed_v1(net, "Mixed_4f", 256, 160, 320, 32, 128, 128)
            net = ep["MaxPool_5a_2x2"] = slim.max_pool2d(net, 2, stride=2, scope="MaxPool_5a_2x2")
            net = ep["Mixed_5b"] = _mixed_v1(net, "Mixed_5b", 256, 160, 320, 32, 128, 128, "Conv2d_0a_3x3")
            net = ep["Mixed_5c"] = _mixed_v1(net, "Mixed_5c", 384, 192, 384, 48, 128, 128)
    return net


def _inception_arg_scope(weight_decay=0.00004, batch_norm_decay=0.9997, batch_norm_epsilon=0.001,
                         batch_norm_scale=False, activation_fn=relu):
    bn = _bn_params(batch_norm_decay, batch_norm_epsilon, batch_norm_scale)
    return [
        ([slim.conv2d, slim.fully_connected], dict(weights_regularizer=slim.l2_regularizer(weight_decay))),
        ([slim.conv2d], dict(weights_initializer=slim.variance_scaling_initializer(), activation_fn=activation_fn,
                             normalizer_fn=slim.batch_norm, normalizer_params=bn)),
        ([slim.batch_norm], bn),
    ]


class _Scopes:
    def __init__(self, lst):
        self.lst = lst
        self.cms = []

    def __enter__(self):
        for ops, kw in self.lst:
            cm = slim.arg_scope(ops, **kw)
            cm.__enter__()
            self.cms.append(cm)

    def __exit__(self, *a):
        for cm in reversed(self.cms):
            cm.__exit__(*a)


def _logits_head(net, num_classes, is_training, keep, pool, scope_pool, scope_drop, scope_logits, spatial_squeeze):
    net = F.avg_pool(net, pool, 1, "VALID") if pool else net
    net = slim.dropout(net, keep, is_training=is_training, scope=scope_drop)
    net = slim.conv2d(net, num_classes, 1, activation_fn=None, normalizer_fn=None, scope=scope_logits)
    return _squeeze(net) if spatial_squeeze else net


def inception_v1(images, num_classes=1000, is_training=True, dropout_keep_prob=0.8, spatial_squeeze=True,
                 scope="InceptionV1", global_pool=False):
    ep = {}
    with _Scopes(_inception_arg_scope()):
        with slim.variable_scope(scope):
            with slim.arg_scope([slim.batch_norm, slim.dropout], is_training=is_training):
                net = inception_v1_base(images, ep)
                if not num_classes:
                    return net, ep
                with slim.variable_scope("Logits"):
                    k = (net.shape[1], net.shape[2]) if global_pool else (7, 7)
                    logits = _logits_head(net, num_classes, is_training, dropout_keep_prob, k, "AvgPool_0a_7x7",
                                          "Dropout_0b", "Conv2d_0c_1x1", spatial_squeeze)
    ep["Logits"] = logits
    return logits, ep


# =============================================================================================
# Inception v2 (vgg/nets/inception_v2.py:29-538), depth_multiplier 1
def inception_v2_base(images, ep, use_separable_conv=True):
    def d(n):
        return n

    with slim.arg_scope([slim.conv2d, slim.max_pool2d, slim.avg_pool2d, slim.separable_conv2d], stride=1,
                        padding="SAME"):
        if use_separable_conv:
            depthwise_multiplier = min(int(d(64) / 3), 8)
            net = slim.separable_conv2d(images, d(64), 7, depth_multiplier=depthwise_multiplier, stride=2,
                                        weights_initializer=slim.trunc_normal(1.0), scope="Conv2d_1a_7x7")
        else:
            net = slim.conv2d(images, d(64), 7, stride=2, weights_initializer=slim.trunc_normal(1.0),
                              scope="Conv2d_1a_7x7")
        ep["Conv2d_1a_7x7"] = net
        net = ep["MaxPool_2a_3x3"] = slim.max_pool2d(net, 3, stride=2, scope="MaxPool_2a_3x3")
        net = ep["Conv2d_2b_1x1"] = slim.conv2d(net, d(64), 1, scope="Conv2d_2b_1x1",
                                                weights_initializer=slim.trunc_normal(0.1))
        net = ep["Conv2d_2c_3x3"] = slim.conv2d(net, d(192), 3, scope="Conv2d_2c_3x3")
        net = ep["MaxPool_3a_3x3"] = slim.max_pool2d(net, 3, stride=2, scope="MaxPool_3a_3x3")

        def mixed(net, name, b0, b1, b2, b3, pool="avg"):
            with slim.variable_scope(name):
                outs = []
                if b0:
                    with slim.variable_scope("Branch_0"):
                        outs.append(slim.conv2d(net, d(b0), 1, scope="Conv2d_0a_1x1"))
                with slim.variable_scope("Branch_1"):
                    x = slim.conv2d(net, d(b1[0]), 1, weights_initializer=slim.trunc_normal(0.09),
                                    scope="Conv2d_0a_1x1")
                    outs.append(slim.conv2d(x, d(b1[1]), 3, scope="Conv2d_0b_3x3"))
                with slim.variable_scope("Branch_2"):
                    x = slim.conv2d(net, d(b2[0]), 1, weights_initializer=slim.trunc_normal(0.09),
                                    scope="Conv2d_0a_1x1")
                    x = slim.conv2d(x, d(b2[1]), 3, scope="Conv2d_0b_3x3")
                    outs.append(slim.conv2d(x, d(b2[1]), 3, scope="Conv2d_0c_3x3"))
                with slim.variable_scope("Branch_3"):
                    x = (slim.avg_pool2d if pool == "avg" else slim.max_pool2d)(
                        net, 3, scope="AvgPool_0a_3x3" if pool == "avg" else "MaxPool_0a_3x3")
                    outs.append(slim.conv2d(x, d(b3), 1, weights_initializer=slim.trunc_normal(0.1),
                                            scope="Conv2d_0b_1x1"))
                return _cat(outs)

        def reduction(net, name, b0, b1):
            with slim.variable_scope(name):
                with slim.variable_scope("Branch_0"):
                    x0 = slim.conv2d(net, d(b0[0]), 1, weights_initializer=slim.trunc_normal(0.09),
                                     scope="Conv2d_0a_1x1")
                    x0 = slim.conv2d(x0, d(b0[1]), 3, stride=2, scope="Conv2d_1a_3x3")
                with slim.variable_scope("Branch_1"):
                    x1 = slim.conv2d(net, d(b1[0]), 1, weights_initializer=slim.trunc_normal(0.09),
                                     scope="Conv2d_0a_1x1")
                    x1 = slim.conv2d(x1, d(b1[1]), 3, scope="Conv2d_0b_3x3")
                    x1 = slim.conv2d(x1, d(b1[1]), 3, stride=2, scope="Conv2d_1a_3x3")
                with slim.variable_scope("Branch_2"):
                    x2 = slim.max_pool2d(net, 3, stride=2, scope="MaxPool_1a_3x3")
                return _cat([x0, x1, x2])

        net = ep["Mixed_3b"] = mixed(net, "Mixed_3b", 64, (64, 64), (64, 96), 32)
        net = ep["Mixed_3c"] = mixed(net, "Mixed_3c", 64, (64, 96), (64, 96), 64)
        net = ep["Mixed_4a"] = reduction(net, "Mixed_4a", (128, 160), (64, 96))
        net = ep["Mixed_4b"] = mixed(net, "Mixed_4b", 224, (64, 96), (96, 128), 128)
        net = ep["Mixed_4c"] = mixed(net, "Mixed_4c", 192, (96, 128), (96, 128), 128)
        net = ep["Mixed_4d"] = mixed(net, "Mixed_4d", 160, (128, 160), (128, 160), 96)
        net = ep["Mixed_4e"] = mixed(net, "Mixed_4e", 96, (128, 192), (160, 192), 96)
        net = ep["Mixed_5a"] = reduction(net, "Mixed_5a", (128, 192), (192, 256))
        net = ep["Mixed_5b"] = mixed(net, "Mixed_5b", 352, (192, 320), (160, 224), 128)
        net = ep["Mixed_5c"] = mixed(net, "Mixed_5c", 352, (192, 320), (192, 224), 128, pool="max")
    return net


def inception_v2(images, num_classes=1000, is_training=True, dropout_keep_prob=0.8, spatial_squeeze=True,
                 scope="InceptionV2", global_pool=False):
    ep = {}
    with _Scopes(_inception_arg_scope()):
        with slim.variable_scope(scope):
            with slim.arg_scope([slim.batch_norm, slim.dropout], is_training=is_training):
                net = inception_v2_base(images, ep)
                if not num_classes:
                    return net, ep
                with slim.variable_scope("Logits"):
                    k = (net.shape[1], net.shape[2]) if global_pool else (min(7, net.shape[1]), min(7, net.shape[2]))
                    logits = _logits_head(net, num_classes, is_training, dropout_keep_prob, k, "AvgPool_1a_7x7",
                                          "Dropout_1b", "Conv2d_1c_1x1", spatial_squeeze)
    ep["Logits"] = logits
    return logits, ep


# =============================================================================================
# Inception v3 (vgg/nets/inception_v3.py:29-555)
def inception_v3_base(images, ep, cifar_variant=False):
    V = "SAME" if cifar_variant else "VALID"  # the reference vgg copy patches every VALID -> SAME
    with slim.arg_scope([slim.conv2d, slim.max_pool2d, slim.avg_pool2d], stride=1, padding=V):
        net = ep["Conv2d_1a_3x3"] = slim.conv2d(images, 32, 3, stride=2, scope="Conv2d_1a_3x3")
        net = ep["Conv2d_2a_3x3"] = slim.conv2d(net, 32, 3, scope="Conv2d_2a_3x3")
        net = ep["Conv2d_2b_3x3"] = slim.conv2d(net, 64, 3, padding="SAME", scope="Conv2d_2b_3x3")
        net = ep["MaxPool_3a_3x3"] = slim.max_pool2d(net, 3, stride=2, scope="MaxPool_3a_3x3")
        net = ep["Conv2d_3b_1x1"] = slim.conv2d(net, 80, 1, scope="Conv2d_3b_1x1")
        net = ep["Conv2d_4a_3x3"] = slim.conv2d(net, 192, 3, scope="Conv2d_4a_3x3")
        net = ep["MaxPool_5a_3x3"] = slim.max_pool2d(net, 3, stride=2, scope="MaxPool_5a_3x3")
    with slim.arg_scope([slim.conv2d, slim.max_pool2d, slim.avg_pool2d], stride=1, padding="SAME"):
        for name, pool_d, b1names in (("Mixed_5b", 32, ("Conv2d_0a_1x1", "Conv2d_0b_5x5")),
                                      ("Mixed_5c", 64, ("Conv2d_0b_1x1", "Conv_1_0c_5x5")),
                                      ("Mixed_5d", 64, ("Conv2d_0a_1x1", "Conv2d_0b_5x5"))):
            with slim.variable_scope(name):
                with slim.variable_scope("Branch_0"):
                    x0 = slim.conv2d(net, 64, 1, scope="Conv2d_0a_1x1")
                with slim.variable_scope("Branch_1"):
                    x1 = slim.conv2d(net, 48, 1, scope=b1names[0])
                    x1 = slim.conv2d(x1, 64, 5, scope=b1names[1])
                with slim.variable_scope("Branch_2"):
                    x2 = slim.conv2d(net, 64, 1, scope="Conv2d_0a_1x1")
                    x2 = slim.conv2d(x2, 96, 3, scope="Conv2d_0b_3x3")
                    x2 = slim.conv2d(x2, 96, 3, scope="Conv2d_0c_3x3")
                with slim.variable_scope("Branch_3"):
                    x3 = slim.avg_pool2d(net, 3, scope="AvgPool_0a_3x3")
                    x3 = slim.conv2d(x3, pool_d, 1, scope="Conv2d_0b_1x1")
                net = ep[name] = _cat([x0, x1, x2, x3])
        with slim.variable_scope("Mixed_6a"):
            with slim.variable_scope("Branch_0"):
                x0 = slim.conv2d(net, 384, 3, stride=2, padding=V, scope="Conv2d_1a_1x1")
            with slim.variable_scope("Branch_1"):
                x1 = slim.conv2d(net, 64, 1, scope="Conv2d_0a_1x1")
                x1 = slim.conv2d(x1, 96, 3, scope="Conv2d_0b_3x3")
                x1 = slim.conv2d(x1, 96, 3, stride=2, padding=V, scope="Conv2d_1a_1x1")
            with slim.variable_scope("Branch_2"):
                x2 = slim.max_pool2d(net, 3, stride=2, padding=V, scope="MaxPool_1a_3x3")
            net = ep["Mixed_6a"] = _cat([x0, x1, x2])
        for name, w in (("Mixed_6b", 128), ("Mixed_6c", 160), ("Mixed_6d", 160), ("Mixed_6e", 192)):
            with slim.variable_scope(name):
                with slim.variable_scope("Branch_0"):
                    x0 = slim.conv2d(net, 192, 1, scope="Conv2d_0a_1x1")
                with slim.variable_scope("Branch_1"):
                    x1 = slim.conv2d(net, w, 1, scope="Conv2d_0a_1x1")
                    x1 = slim.conv2d(x1, w, (1, 7), scope="Conv2d_0b_1x7")
                    x1 = slim.conv2d(x1, 192, (7, 1), scope="Conv2d_0c_7x1")
                with slim.variable_scope("Branch_2"):
                    x2 = slim.conv2d(net, w, 1, scope="Conv2d_0a_1x1")
                    x2 = slim.conv2d(x2, w, (7, 1), scope="Conv2d_0b_7x1")
                    x2 = slim.conv2d(x2, w, (1, 7), scope="Conv2d_0c_1x7")
                    x2 = slim.conv2d(x2, w, (7, 1), scope="Conv2d_0d_7x1")
                    x2 = slim.conv2d(x2, 192, (1, 7), scope="Conv2d_0e_1x7")
                with slim.variable_scope("Branch_3"):
                    x3 = slim.avg_pool2d(net, 3, scope="AvgPool_0a_3x3")
                    x3 = slim.conv2d(x3, 192, 1, scope="Conv2d_0b_1x1")
                net = ep[name] = _cat([x0, x1, x2, x3])
        with slim.variable_scope("Mixed_7a"):
            with slim.variable_scope("Branch_0"):
                x0 = slim.conv2d(net, 192, 1, scope="Conv2d_0a_1x1")
                x0 = slim.conv2d(x0, 320, 3, stride=2, padding=V, scope="Conv2d_1a_3x3")
            with slim.variable_scope("Branch_1"):
                x1 = slim.conv2d(net, 192, 1, scope="Conv2d_0a_1x1")
                x1 = slim.conv2d(x1, 192, (1, 7), scope="Conv2d_0b_1x7")
                x1 = slim.conv2d(x1, 192, (7, 1), scope="Conv2d_0c_7x1")
                x1 = slim.conv2d(x1, 192, 3, stride=2, padding=V, scope="Conv2d_1a_3x3")
            with slim.variable_scope("Branch_2"):
                x2 = slim.max_pool2d(net, 3, stride=2, padding=V, scope="MaxPool_1a_3x3")
            net = ep["Mixed_7a"] = _cat([x0, x1, x2])
        for name, b1c in (("Mixed_7b", "Conv2d_0b_3x1"), ("Mixed_7c", "Conv2d_0c_3x1")):
            with slim.variable_scope(name):
                with slim.variable_scope("Branch_0"):
                    x0 = slim.conv2d(net, 320, 1, scope="Conv2d_0a_1x1")
                with slim.variable_scope("Branch_1"):
                    x1 = slim.conv2d(net, 384, 1, scope="Conv2d_0a_1x1")
                    x1 = _cat([slim.conv2d(x1, 384, (1, 3), scope="Conv2d_0b_1x3"),
                               slim.conv2d(x1, 384, (3, 1), scope=b1c)])
                with slim.variable_scope("Branch_2"):
                    x2 = slim.conv2d(net, 448, 1, scope="Conv2d_0a_1x1")
                    x2 = slim.conv2d(x2, 384, 3, scope="Conv2d_0b_3x3")
                    x2 = _cat([slim.conv2d(x2, 384, (1, 3), scope="Conv2d_0c_1x3"),
                               slim.conv2d(x2, 384, (3, 1), scope="Conv2d_0d_3x1")])
                with slim.variable_scope("Branch_3"):
                    x3 = slim.avg_pool2d(net, 3, scope="AvgPool_0a_3x3")
                    x3 = slim.conv2d(x3, 192, 1, scope="Conv2d_0b_1x1")
                net = ep[name] = _cat([x0, x1, x2, x3])
    return net


def inception_v3(images, num_classes=1000, is_training=True, dropout_keep_prob=0.8, spatial_squeeze=True,
                 scope="InceptionV3", create_aux_logits=True, cifar_variant=False, global_pool=False):
    ep = {}
    with _Scopes(_inception_arg_scope()):
        with slim.variable_scope(scope):
            with slim.arg_scope([slim.batch_norm, slim.dropout], is_training=is_training):
                net = inception_v3_base(images, ep, cifar_variant)
                if not num_classes:
                    return net, ep
                aux = None
                with slim.arg_scope([slim.conv2d, slim.max_pool2d, slim.avg_pool2d], stride=1, padding="SAME"):
                    if create_aux_logits:
                        with slim.variable_scope("AuxLogits"):
                            a = F.avg_pool(ep["Mixed_6e"], 5, 3, "VALID")
                            a = slim.conv2d(a, 128, 1, scope="Conv2d_1b_1x1")
                            k = (a.shape[1], a.shape[2])
                            a = slim.conv2d(a, 768, k, weights_initializer=slim.trunc_normal(0.01), padding="VALID",
                                            scope="Conv2d_2a_%dx%d" % k)
                            a = slim.conv2d(a, num_classes, 1, activation_fn=None, normalizer_fn=None,
                                            weights_initializer=slim.trunc_normal(0.001), scope="Conv2d_2b_1x1")
                            aux = ep["AuxLogits"] = _squeeze(a) if spatial_squeeze else a
                    with slim.variable_scope("Logits"):
                        k = (net.shape[1], net.shape[2])
                        logits = _logits_head(net, num_classes, is_training, dropout_keep_prob, k,
                                              "AvgPool_1a_%dx%d" % k, "Dropout_1b", "Conv2d_1c_1x1", spatial_squeeze)
    ep["Logits"] = logits
    if is_training and aux is not None:
        return (logits, aux), ep
    return logits, ep


# =============================================================================================
# MobileNet v1 (vgg/nets/mobilenet_v1.py:120-472)
MOBILENET_V1_CONV_DEFS = [("conv", 3, 2, 32)] + [("sep", 3, s, d) for s, d in (
    (1, 64), (2, 128), (1, 128), (2, 256), (1, 256), (2, 512), (1, 512), (1, 512), (1, 512), (1, 512), (1, 512),
    (2, 1024), (1, 1024))]


def mobilenet_v1_base(images, ep, depth_multiplier=1.0, min_depth=8):
    def depth(d):
        return max(int(d * depth_multiplier), min_depth)

    net = images
    with slim.arg_scope([slim.conv2d, slim.separable_conv2d], padding="SAME"):
        for i, (kind, k, s, d) in enumerate(MOBILENET_V1_CONV_DEFS):
            if kind == "conv":
                name = "Conv2d_%d" % i
                net = ep[name] = slim.conv2d(net, depth(d), k, stride=s, scope=name)
            else:
                name = "Conv2d_%d_depthwise" % i
                net = ep[name] = slim.separable_conv2d(net, None, k, depth_multiplier=1, stride=s, scope=name)
                name = "Conv2d_%d_pointwise" % i
                net = ep[name] = slim.conv2d(net, depth(d), 1, stride=1, scope=name)
    return net


def mobilenet_v1(images, num_classes=1000, is_training=True, dropout_keep_prob=0.999, depth_multiplier=1.0,
                 min_depth=8, spatial_squeeze=True, scope="MobilenetV1", global_pool=False, weight_decay=0.00004):
    ep = {}
    bn = dict(decay=0.9997, epsilon=0.001, scale=True, center=True)
    with slim.arg_scope([slim.conv2d, slim.separable_conv2d], weights_initializer=slim.trunc_normal(0.09),
                        activation_fn=_relu6, normalizer_fn=slim.batch_norm, normalizer_params=bn):
        with slim.arg_scope([slim.batch_norm], is_training=is_training, **bn), \
                slim.arg_scope([slim.conv2d], weights_regularizer=slim.l2_regularizer(weight_decay)):
            with slim.variable_scope(scope):
                net = mobilenet_v1_base(images, ep, depth_multiplier, min_depth)
                if not num_classes:
                    return net, ep
                with slim.variable_scope("Logits"):
                    k = (net.shape[1], net.shape[2]) if global_pool else (min(7, net.shape[1]), min(7, net.shape[2]))
                    logits = _logits_head(net, num_classes, is_training, dropout_keep_prob, k, "AvgPool_1a",
                                          "Dropout_1b", "Conv2d_1c_1x1", spatial_squeeze)
    ep["Logits"] = logits
    return logits, ep


# =============================================================================================
# MobileNet v2 (vgg/nets/mobilenet/mobilenet_v2.py V2_DEF, conv_blocks.expanded_conv)
MOBILENET_V2_DEF = [(1, 16, 1, 1), (6, 24, 2, 2), (6, 32, 3, 2), (6, 64, 4, 2), (6, 96, 3, 1), (6, 160, 3, 2),
                    (6, 320, 1, 1)]


def _make_divisible(v, divisor=8, min_value=None):
    min_value = min_value or divisor
    new_v = max(min_value, int(v + divisor / 2) // divisor * divisor)
    if new_v < 0.9 * v:
        new_v += divisor
    return new_v


def mobilenet_v2(images, num_classes=1001, is_training=True, depth_multiplier=1.0, scope="MobilenetV2",
                 dropout_keep_prob=0.8, finegrain_classification_mode=False, spatial_squeeze=True,
                 weight_decay=0.00004):
    ep = {}
    bn = dict(decay=0.997, epsilon=0.001, scale=True, center=True)

    def dm(d):
        return _make_divisible(d * depth_multiplier, 8)

    with slim.arg_scope([slim.conv2d, slim.separable_conv2d], normalizer_fn=slim.batch_norm, normalizer_params=bn,
                        activation_fn=_relu6, weights_initializer=slim.trunc_normal(0.09)), \
            slim.arg_scope([slim.batch_norm], is_training=is_training, **bn), \
            slim.arg_scope([slim.conv2d], weights_regularizer=slim.l2_regularizer(weight_decay)):
        with slim.variable_scope(scope):
            net = ep["layer_1"] = slim.conv2d(images, dm(32), 3, stride=2, scope="Conv")
            layer = 1
            cin = dm(32)
            for t, c, n, s in MOBILENET_V2_DEF:
                for i in range(n):
                    stride = s if i == 0 else 1
                    name = "expanded_conv" if layer == 1 else "expanded_conv_%d" % (layer - 1)
                    out = dm(c)
                    with slim.variable_scope(name):
                        x = net
                        if t != 1:
                            x = slim.conv2d(x, _make_divisible(cin * t, 8), 1, scope="expand")
                        x = ep["layer_%d/depthwise_output" % (layer + 1)] = slim.separable_conv2d(
                            x, None, 3, depth_multiplier=1, stride=stride, scope="depthwise")
                        x = slim.conv2d(x, out, 1, activation_fn=None, scope="project")
                        if stride == 1 and cin == out:
                            x = as_tensor(x) + as_tensor(net)
                    net = ep["layer_%d" % (layer + 1)] = x
                    cin = out
                    layer += 1
            last = 1280 if not finegrain_classification_mode and depth_multiplier < 1 else dm(1280)
            net = slim.conv2d(net, max(1280, last) if depth_multiplier < 1 else dm(1280), 1,
                              scope="Conv_1")
            if not num_classes:
                return net, ep
            with slim.variable_scope("Logits"):
                net = F.global_avg_pool(net).reshape(net.shape[0], 1, 1, -1)
                net = slim.dropout(net, dropout_keep_prob, is_training=is_training, scope="Dropout")
                logits = slim.conv2d(net, num_classes, 1, activation_fn=None, normalizer_fn=None,
                                     biases_initializer=("constant", 0.0), scope="Conv2d_1c_1x1")
                logits = _squeeze(logits) if spatial_squeeze else logits
    ep["Logits"] = logits
    return logits, ep
