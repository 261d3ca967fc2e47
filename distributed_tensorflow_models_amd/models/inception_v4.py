"""Inception-v4 and Inception-ResNet-v2 on the functional slim facade (Szegedy et al. 2016).

Structure, endpoint and variable names follow the reference slim definitions
(reference vgg/nets/inception_v4.py:34-337, vgg/nets/inception_resnet_v2.py:32-398); the
reference tests' golden shapes are checked in tests/test_models.py.  Every conv is the fused
conv+BN(+ReLU) HIP path on the GPU (BatchNorm without gamma: ``scale=False`` as in
inception_utils.inception_arg_scope); the residual ``net + scale * up`` of the Inception-ResNet
blocks is a single fused elementwise pass over the materialised tensors.
"""
import torch

from ..compat import slim
from ..ops import nn as F
from ..ops.lazy import as_tensor
from .slim_nets import _cat, _Scopes, _inception_arg_scope

relu = torch.relu


def _conv(x, n, k, scope, **kw):
    return slim.conv2d(x, n, k, scope=scope, **kw)


# ---------------------------------------------------------------------------------------------
# Inception-v4 blocks
def block_inception_a(x, scope):
    with slim.variable_scope(scope):
        with slim.variable_scope("Branch_0"):
            b0 = _conv(x, 96, 1, "Conv2d_0a_1x1")
        with slim.variable_scope("Branch_1"):
            b1 = _conv(_conv(x, 64, 1, "Conv2d_0a_1x1"), 96, 3, "Conv2d_0b_3x3")
        with slim.variable_scope("Branch_2"):
            b2 = _conv(x, 64, 1, "Conv2d_0a_1x1")
            b2 = _conv(_conv(b2, 96, 3, "Conv2d_0b_3x3"), 96, 3, "Conv2d_0c_3x3")
        with slim.variable_scope("Branch_3"):
            b3 = _conv(slim.avg_pool2d(x, 3, scope="AvgPool_0a_3x3"), 96, 1, "Conv2d_0b_1x1")
        return _cat([b0, b1, b2, b3])


def block_reduction_a(x, scope):
    with slim.variable_scope(scope):
        with slim.variable_scope("Branch_0"):
            b0 = _conv(x, 384, 3, "Conv2d_1a_3x3", stride=2, padding="VALID")
        with slim.variable_scope("Branch_1"):
            b1 = _conv(_conv(x, 192, 1, "Conv2d_0a_1x1"), 224, 3, "Conv2d_0b_3x3")
            b1 = _conv(b1, 256, 3, "Conv2d_1a_3x3", stride=2, padding="VALID")
        with slim.variable_scope("Branch_2"):
            b2 = slim.max_pool2d(x, 3, stride=2, padding="VALID", scope="MaxPool_1a_3x3")
        return _cat([b0, b1, b2])


def block_inception_b(x, scope):
    with slim.variable_scope(scope):
        with slim.variable_scope("Branch_0"):
            b0 = _conv(x, 384, 1, "Conv2d_0a_1x1")
        with slim.variable_scope("Branch_1"):
            b1 = _conv(x, 192, 1, "Conv2d_0a_1x1")
            b1 = _conv(_conv(b1, 224, (1, 7), "Conv2d_0b_1x7"), 256, (7, 1), "Conv2d_0c_7x1")
        with slim.variable_scope("Branch_2"):
            b2 = _conv(x, 192, 1, "Conv2d_0a_1x1")
            for n, k, nm in ((192, (7, 1), "Conv2d_0b_7x1"), (224, (1, 7), "Conv2d_0c_1x7"),
                             (224, (7, 1), "Conv2d_0d_7x1"), (256, (1, 7), "Conv2d_0e_1x7")):
                b2 = _conv(b2, n, k, nm)
        with slim.variable_scope("Branch_3"):
            b3 = _conv(slim.avg_pool2d(x, 3, scope="AvgPool_0a_3x3"), 128, 1, "Conv2d_0b_1x1")
        return _cat([b0, b1, b2, b3])


def block_reduction_b(x, scope):
    with slim.variable_scope(scope):
        with slim.variable_scope("Branch_0"):
            b0 = _conv(_conv(x, 192, 1, "Conv2d_0a_1x1"), 192, 3, "Conv2d_1a_3x3", stride=2, padding="VALID")
        with slim.variable_scope("Branch_1"):
            b1 = _conv(x, 256, 1, "Conv2d_0a_1x1")
            b1 = _conv(_conv(b1, 256, (1, 7), "Conv2d_0b_1x7"), 320, (7, 1), "Conv2d_0c_7x1")
            b1 = _conv(b1, 320, 3, "Conv2d_1a_3x3", stride=2, padding="VALID")
        with slim.variable_scope("Branch_2"):
            b2 = slim.max_pool2d(x, 3, stride=2, padding="VALID", scope="MaxPool_1a_3x3")
        return _cat([b0, b1, b2])


def block_inception_c(x, scope):
    with slim.variable_scope(scope):
        with slim.variable_scope("Branch_0"):
            b0 = _conv(x, 256, 1, "Conv2d_0a_1x1")
        with slim.variable_scope("Branch_1"):
            b1 = _conv(x, 384, 1, "Conv2d_0a_1x1")
            b1 = _cat([_conv(b1, 256, (1, 3), "Conv2d_0b_1x3"), _conv(b1, 256, (3, 1), "Conv2d_0c_3x1")])
        with slim.variable_scope("Branch_2"):
            b2 = _conv(x, 384, 1, "Conv2d_0a_1x1")
            b2 = _conv(_conv(b2, 448, (3, 1), "Conv2d_0b_3x1"), 512, (1, 3), "Conv2d_0c_1x3")
            b2 = _cat([_conv(b2, 256, (1, 3), "Conv2d_0d_1x3"), _conv(b2, 256, (3, 1), "Conv2d_0e_3x1")])
        with slim.variable_scope("Branch_3"):
            b3 = _conv(slim.avg_pool2d(x, 3, scope="AvgPool_0a_3x3"), 256, 1, "Conv2d_0b_1x1")
        return _cat([b0, b1, b2, b3])


V4_ENDPOINTS = ["Conv2d_1a_3x3", "Conv2d_2a_3x3", "Conv2d_2b_3x3", "Mixed_3a", "Mixed_4a", "Mixed_5a", "Mixed_5b",
                "Mixed_5c", "Mixed_5d", "Mixed_5e", "Mixed_6a", "Mixed_6b", "Mixed_6c", "Mixed_6d", "Mixed_6e",
                "Mixed_6f", "Mixed_6g", "Mixed_6h", "Mixed_7a", "Mixed_7b", "Mixed_7c", "Mixed_7d"]


def inception_v4_base(images, ep, final_endpoint="Mixed_7d"):
    if final_endpoint not in V4_ENDPOINTS:
        raise ValueError("Unknown final endpoint %s" % final_endpoint)

    def done(name, net):
        ep[name] = net
        return name == final_endpoint

    with slim.arg_scope([slim.conv2d, slim.max_pool2d, slim.avg_pool2d], stride=1, padding="SAME"):
        net = _conv(images, 32, 3, "Conv2d_1a_3x3", stride=2, padding="VALID")
        if done("Conv2d_1a_3x3", net):
            return net
        net = _conv(net, 32, 3, "Conv2d_2a_3x3", padding="VALID")
        if done("Conv2d_2a_3x3", net):
            return net
        net = _conv(net, 64, 3, "Conv2d_2b_3x3")
        if done("Conv2d_2b_3x3", net):
            return net
        with slim.variable_scope("Mixed_3a"):
            with slim.variable_scope("Branch_0"):
                b0 = slim.max_pool2d(net, 3, stride=2, padding="VALID", scope="MaxPool_0a_3x3")
            with slim.variable_scope("Branch_1"):
                b1 = _conv(net, 96, 3, "Conv2d_0a_3x3", stride=2, padding="VALID")
            net = _cat([b0, b1])
        if done("Mixed_3a", net):
            return net
        with slim.variable_scope("Mixed_4a"):
            with slim.variable_scope("Branch_0"):
                b0 = _conv(_conv(net, 64, 1, "Conv2d_0a_1x1"), 96, 3, "Conv2d_1a_3x3", padding="VALID")
            with slim.variable_scope("Branch_1"):
                b1 = _conv(net, 64, 1, "Conv2d_0a_1x1")
                b1 = _conv(_conv(b1, 64, (1, 7), "Conv2d_0b_1x7"), 64, (7, 1), "Conv2d_0c_7x1")
                b1 = _conv(b1, 96, 3, "Conv2d_1a_3x3", padding="VALID")
            net = _cat([b0, b1])
        if done("Mixed_4a", net):
            return net
        with slim.variable_scope("Mixed_5a"):
            with slim.variable_scope("Branch_0"):
                b0 = _conv(net, 192, 3, "Conv2d_1a_3x3", stride=2, padding="VALID")
            with slim.variable_scope("Branch_1"):
                b1 = slim.max_pool2d(net, 3, stride=2, padding="VALID", scope="MaxPool_1a_3x3")
            net = _cat([b0, b1])
        if done("Mixed_5a", net):
            return net
        for block, prefix, n, red in ((block_inception_a, "Mixed_5", 4, (block_reduction_a, "Mixed_6a")),
                                      (block_inception_b, "Mixed_6", 7, (block_reduction_b, "Mixed_7a")),
                                      (block_inception_c, "Mixed_7", 3, None)):
            for i in range(n):
                name = prefix + chr(ord("b") + i)
                net = block(net, name)
                if done(name, net):
                    return net
            if red is not None:
                net = red[0](net, red[1])
                if done(red[1], net):
                    return net
    raise ValueError("Unknown final endpoint %s" % final_endpoint)


def _fc_head(net, num_classes, scope):
    return slim.fully_connected(slim.flatten(net), num_classes, activation_fn=None, scope=scope)


def inception_v4(images, num_classes=1001, is_training=True, dropout_keep_prob=0.8, scope="InceptionV4",
                 create_aux_logits=True, final_endpoint="Mixed_7d"):
    ep = {}
    aux = None
    with _Scopes(_inception_arg_scope()):
        with slim.variable_scope(scope):
            with slim.arg_scope([slim.batch_norm, slim.dropout], is_training=is_training):
                net = inception_v4_base(images, ep, final_endpoint)
                if final_endpoint != "Mixed_7d":
                    return net, ep
                with slim.arg_scope([slim.conv2d, slim.max_pool2d, slim.avg_pool2d], stride=1, padding="SAME"):
                    if create_aux_logits and num_classes:
                        with slim.variable_scope("AuxLogits"):
                            a = slim.avg_pool2d(ep["Mixed_6h"], 5, stride=3, padding="VALID", scope="AvgPool_1a_5x5")
                            a = _conv(a, 128, 1, "Conv2d_1b_1x1")
                            a = _conv(a, 768, (a.shape[1], a.shape[2]), "Conv2d_2a", padding="VALID")
                            aux = ep["AuxLogits"] = _fc_head(a, num_classes, "Aux_logits")
                    with slim.variable_scope("Logits"):
                        k = (as_tensor(net).shape[1], as_tensor(net).shape[2])
                        net = ep["global_pool"] = slim.avg_pool2d(net, k, padding="VALID", scope="AvgPool_1a")
                        if not num_classes:
                            return net, ep
                        net = slim.dropout(net, dropout_keep_prob, scope="Dropout_1b")
                        net = ep["PreLogitsFlatten"] = slim.flatten(net, scope="PreLogitsFlatten")
                        logits = ep["Logits"] = slim.fully_connected(net, num_classes, activation_fn=None,
                                                                     scope="Logits")
                        ep["Predictions"] = torch.softmax(as_tensor(logits).float(), -1)
    if is_training and aux is not None:
        return (logits, aux), ep
    return logits, ep


# ---------------------------------------------------------------------------------------------
# Inception-ResNet-v2 blocks: net + scale * conv1x1(concat(branches)), then activation
def _residual(net, up, scale, activation_fn):
    out = as_tensor(net) + as_tensor(up) * scale
    return activation_fn(out) if activation_fn is not None else out


def block35(net, scale=1.0, activation_fn=relu, scope=None):
    with slim.variable_scope(scope, default_name="Block35"):
        with slim.variable_scope("Branch_0"):
            b0 = _conv(net, 32, 1, "Conv2d_1x1")
        with slim.variable_scope("Branch_1"):
            b1 = _conv(_conv(net, 32, 1, "Conv2d_0a_1x1"), 32, 3, "Conv2d_0b_3x3")
        with slim.variable_scope("Branch_2"):
            b2 = _conv(net, 32, 1, "Conv2d_0a_1x1")
            b2 = _conv(_conv(b2, 48, 3, "Conv2d_0b_3x3"), 64, 3, "Conv2d_0c_3x3")
        up = _conv(_cat([b0, b1, b2]), as_tensor(net).shape[-1], 1, "Conv2d_1x1", normalizer_fn=None,
                   activation_fn=None)
        return _residual(net, up, scale, activation_fn)


def block17(net, scale=1.0, activation_fn=relu, scope=None):
    with slim.variable_scope(scope, default_name="Block17"):
        with slim.variable_scope("Branch_0"):
            b0 = _conv(net, 192, 1, "Conv2d_1x1")
        with slim.variable_scope("Branch_1"):
            b1 = _conv(net, 128, 1, "Conv2d_0a_1x1")
            b1 = _conv(_conv(b1, 160, (1, 7), "Conv2d_0b_1x7"), 192, (7, 1), "Conv2d_0c_7x1")
        up = _conv(_cat([b0, b1]), as_tensor(net).shape[-1], 1, "Conv2d_1x1", normalizer_fn=None, activation_fn=None)
        return _residual(net, up, scale, activation_fn)


def block8(net, scale=1.0, activation_fn=relu, scope=None):
    with slim.variable_scope(scope, default_name="Block8"):
        with slim.variable_scope("Branch_0"):
            b0 = _conv(net, 192, 1, "Conv2d_1x1")
        with slim.variable_scope("Branch_1"):
            b1 = _conv(net, 192, 1, "Conv2d_0a_1x1")
            b1 = _conv(_conv(b1, 224, (1, 3), "Conv2d_0b_1x3"), 256, (3, 1), "Conv2d_0c_3x1")
        up = _conv(_cat([b0, b1]), as_tensor(net).shape[-1], 1, "Conv2d_1x1", normalizer_fn=None, activation_fn=None)
        return _residual(net, up, scale, activation_fn)


def inception_resnet_v2_base(images, ep, final_endpoint="Conv2d_7b_1x1", align_feature_maps=False,
                             activation_fn=relu, output_stride=16):
    if output_stride not in (8, 16):
        raise ValueError("output_stride must be 8 or 16.")
    pad = "SAME" if align_feature_maps else "VALID"
    s6 = 1 if output_stride == 8 else 2  # atrous: keep 35x35 (well, 33x33) resolution after Mixed_6a

    def done(name, net):
        ep[name] = net
        return name == final_endpoint

    with slim.arg_scope([slim.conv2d, slim.max_pool2d, slim.avg_pool2d], stride=1, padding="SAME"):
        net = _conv(images, 32, 3, "Conv2d_1a_3x3", stride=2, padding=pad)
        if done("Conv2d_1a_3x3", net):
            return net
        net = _conv(net, 32, 3, "Conv2d_2a_3x3", padding=pad)
        if done("Conv2d_2a_3x3", net):
            return net
        net = _conv(net, 64, 3, "Conv2d_2b_3x3")
        if done("Conv2d_2b_3x3", net):
            return net
        net = slim.max_pool2d(net, 3, stride=2, padding=pad, scope="MaxPool_3a_3x3")
        if done("MaxPool_3a_3x3", net):
            return net
        net = _conv(net, 80, 1, "Conv2d_3b_1x1", padding=pad)
        if done("Conv2d_3b_1x1", net):
            return net
        net = _conv(net, 192, 3, "Conv2d_4a_3x3", padding=pad)
        if done("Conv2d_4a_3x3", net):
            return net
        net = slim.max_pool2d(net, 3, stride=2, padding=pad, scope="MaxPool_5a_3x3")
        if done("MaxPool_5a_3x3", net):
            return net
        with slim.variable_scope("Mixed_5b"):
            with slim.variable_scope("Branch_0"):
                b0 = _conv(net, 96, 1, "Conv2d_1x1")
            with slim.variable_scope("Branch_1"):
                b1 = _conv(_conv(net, 48, 1, "Conv2d_0a_1x1"), 64, 5, "Conv2d_0b_5x5")
            with slim.variable_scope("Branch_2"):
                b2 = _conv(net, 64, 1, "Conv2d_0a_1x1")
                b2 = _conv(_conv(b2, 96, 3, "Conv2d_0b_3x3"), 96, 3, "Conv2d_0c_3x3")
            with slim.variable_scope("Branch_3"):
                b3 = slim.avg_pool2d(net, 3, stride=1, padding="SAME", scope="AvgPool_0a_3x3")
                b3 = _conv(b3, 64, 1, "Conv2d_0b_1x1")
            net = _cat([b0, b1, b2, b3])
        if done("Mixed_5b", net):
            return net
        net = slim.repeat(net, 10, block35, scale=0.17, activation_fn=activation_fn)
        with slim.variable_scope("Mixed_6a"):
            with slim.variable_scope("Branch_0"):
                b0 = _conv(net, 384, 3, "Conv2d_1a_3x3", stride=s6, padding=pad)
            with slim.variable_scope("Branch_1"):
                b1 = _conv(_conv(net, 256, 1, "Conv2d_0a_1x1"), 256, 3, "Conv2d_0b_3x3")
                b1 = _conv(b1, 384, 3, "Conv2d_1a_3x3", stride=s6, padding=pad)
            with slim.variable_scope("Branch_2"):
                b2 = slim.max_pool2d(net, 3, stride=s6, padding=pad, scope="MaxPool_1a_3x3")
            net = _cat([b0, b1, b2])
        if done("Mixed_6a", net):
            return net
        with slim.arg_scope([slim.conv2d], rate=2 if output_stride == 8 else 1):
            net = slim.repeat(net, 20, block17, scale=0.10, activation_fn=activation_fn)
        if done("PreAuxLogits", net):
            return net
        if output_stride == 8:
            raise ValueError("output_stride==8 is only supported up to the PreAuxlogits end_point for now.")
        with slim.variable_scope("Mixed_7a"):
            with slim.variable_scope("Branch_0"):
                b0 = _conv(_conv(net, 256, 1, "Conv2d_0a_1x1"), 384, 3, "Conv2d_1a_3x3", stride=2, padding=pad)
            with slim.variable_scope("Branch_1"):
                b1 = _conv(_conv(net, 256, 1, "Conv2d_0a_1x1"), 288, 3, "Conv2d_1a_3x3", stride=2, padding=pad)
            with slim.variable_scope("Branch_2"):
                b2 = _conv(_conv(net, 256, 1, "Conv2d_0a_1x1"), 288, 3, "Conv2d_0b_3x3")
                b2 = _conv(b2, 320, 3, "Conv2d_1a_3x3", stride=2, padding=pad)
            with slim.variable_scope("Branch_3"):
                b3 = slim.max_pool2d(net, 3, stride=2, padding=pad, scope="MaxPool_1a_3x3")
            net = _cat([b0, b1, b2, b3])
        if done("Mixed_7a", net):
            return net
        net = slim.repeat(net, 9, block8, scale=0.20, activation_fn=activation_fn)
        net = block8(net, activation_fn=None)
        net = _conv(net, 1536, 1, "Conv2d_7b_1x1")
        if done("Conv2d_7b_1x1", net):
            return net
    raise ValueError("final_endpoint (%s) not recognized" % final_endpoint)


def inception_resnet_v2(images, num_classes=1001, is_training=True, dropout_keep_prob=0.8,
                        scope="InceptionResnetV2", create_aux_logits=True, activation_fn=relu,
                        weight_decay=0.00004):
    ep = {}
    aux = None
    bn = dict(decay=0.9997, epsilon=0.001, scale=False)
    with slim.arg_scope([slim.conv2d, slim.fully_connected], weights_regularizer=slim.l2_regularizer(weight_decay),
                        biases_regularizer=slim.l2_regularizer(weight_decay)), \
            slim.arg_scope([slim.conv2d], activation_fn=activation_fn, normalizer_fn=slim.batch_norm,
                           normalizer_params=bn), slim.arg_scope([slim.batch_norm], **bn):
        with slim.variable_scope(scope):
            with slim.arg_scope([slim.batch_norm, slim.dropout], is_training=is_training):
                net = inception_resnet_v2_base(images, ep, activation_fn=activation_fn)
                if create_aux_logits and num_classes:
                    with slim.variable_scope("AuxLogits"):
                        a = slim.avg_pool2d(ep["PreAuxLogits"], 5, stride=3, padding="VALID", scope="Conv2d_1a_3x3")
                        a = _conv(a, 128, 1, "Conv2d_1b_1x1")
                        a = _conv(a, 768, (a.shape[1], a.shape[2]), "Conv2d_2a_5x5", padding="VALID")
                        aux = ep["AuxLogits"] = _fc_head(a, num_classes, "Logits")
                with slim.variable_scope("Logits"):
                    t = as_tensor(net)
                    net = ep["global_pool"] = slim.avg_pool2d(t, (t.shape[1], t.shape[2]), padding="VALID",
                                                              scope="AvgPool_1a_8x8")
                    if not num_classes:
                        return net, ep
                    net = slim.dropout(slim.flatten(net), dropout_keep_prob, is_training=is_training, scope="Dropout")
                    ep["PreLogitsFlatten"] = net
                    logits = ep["Logits"] = slim.fully_connected(net, num_classes, activation_fn=None, scope="Logits")
                    ep["Predictions"] = torch.softmax(as_tensor(logits).float(), -1)
    if is_training and aux is not None:
        return (logits, aux), ep
    return logits, ep
