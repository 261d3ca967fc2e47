"""Classic CNNs of the reference zoo (NHWC, TF variable names):

* ``cifar10_cnn``  - the TF CIFAR-10 tutorial model  (reference cnn/cifar10.py:203-282)
* ``lenet``        - vgg/nets/lenet.py:26-97
* ``cifarnet``     - vgg/nets/cifarnet.py:28-117 / cifarnet/cifarnet.py:28-118 (patched copy returns
                     softmax; here logits, ``compat_double_softmax=True`` reproduces the defect)
* ``alexnet_v2``   - alexnet/alexnet.py:45-142 (CIFAR branch: stride-1 conv1 when num_classes==10;
                     fc6 as a 5x5 'SAME' conv)
* ``vgg_a/16/19``  - vgg/nets/vgg.py:49-302 (``fc_conv_padding``; the vgg copy forces 'same' for
                     vgg_16, vgg/nets/vgg.py:202 -> ``cifar_variant``)
* ``overfeat``     - vgg/nets/overfeat.py:40-131
"""
import torch

from ..ops import nn as F
from ..ops import reference as R
from ..ops.lrn import lrn
from .layers import Conv2d, Dropout, FullyConnected, Layer, _join


def _flatten(x):
    from ..ops.lazy import as_tensor
    x = as_tensor(x)
    return x.reshape(x.shape[0], -1)


class Cifar10CNN(Layer):
    """cnn/cifar10.py inference(): conv1-pool1-norm1-conv2-norm2-pool2-local3-local4-softmax_linear.
    Weight decay: local3/local4 0.004 (cifar10.py:262-279); conv layers 0."""
    default_image_size = 24

    def __init__(self, num_classes=10, image_size=24, scope=""):
        super().__init__(scope)
        self.conv1 = Conv2d(_join(scope, "conv1"), 3, 64, 5, 1, "SAME", "relu", None, True, 0.0,
                            ("truncated_normal", 5e-2), 0.0)
        self.conv2 = Conv2d(_join(scope, "conv2"), 64, 64, 5, 1, "SAME", "relu", None, True, 0.0,
                            ("truncated_normal", 5e-2), 0.1)
        s = image_size
        for _ in range(2):
            s = -(-s // 2)
        dim = s * s * 64
        self.local3 = FullyConnected(_join(scope, "local3"), dim, 384, "relu", None, True, 0.004,
                                     ("truncated_normal", 0.04), 0.1)
        self.local4 = FullyConnected(_join(scope, "local4"), 384, 192, "relu", None, True, 0.004,
                                     ("truncated_normal", 0.04), 0.1)
        self.softmax_linear = FullyConnected(_join(scope, "softmax_linear"), 192, num_classes, None, None, True, 0.0,
                                             ("truncated_normal", 1 / 192.0), 0.0)

    def forward(self, x, training=True, end_points=None):
        net = self.conv1(x, training)
        net = F.max_pool(net, 3, 2, "SAME")
        net = lrn(net, 4, 1.0, 0.001 / 9.0, 0.75)
        net = self.conv2(net, training)
        net = lrn(net, 4, 1.0, 0.001 / 9.0, 0.75)
        net = F.max_pool(net, 3, 2, "SAME")
        net = self.local3(_flatten(net), training)
        net = self.local4(net, training)
        return self.softmax_linear(net, training)


class LeNet(Layer):
    default_image_size = 28

    def __init__(self, num_classes=10, dropout_keep_prob=0.5, weight_decay=0.0, scope="LeNet", in_channels=1):
        super().__init__(scope)
        init = ("truncated_normal", 0.1)
        self.conv1 = Conv2d(_join(scope, "conv1"), in_channels, 32, 5, 1, "SAME", "relu", None, True, weight_decay, init)
        self.conv2 = Conv2d(_join(scope, "conv2"), 32, 64, 5, 1, "SAME", "relu", None, True, weight_decay, init)
        self.fc3 = FullyConnected(_join(scope, "fc3"), 7 * 7 * 64, 1024, "relu", None, True, weight_decay, init)
        self.dropout3 = Dropout(_join(scope, "dropout3"), dropout_keep_prob)
        self.fc4 = FullyConnected(_join(scope, "fc4"), 1024, num_classes, None, None, True, weight_decay, init) \
            if num_classes else None

    def forward(self, x, training=True, end_points=None):
        net = F.max_pool(self.conv1(x, training), 2, 2, "VALID")
        net = F.max_pool(self.conv2(net, training), 2, 2, "VALID")
        net = self.fc3(_flatten(net), training)
        if self.fc4 is None:
            return net
        net = self.dropout3(net, training)
        return self.fc4(net, training)


class CifarNet(Layer):
    default_image_size = 32

    def __init__(self, num_classes=10, dropout_keep_prob=0.5, weight_decay=0.004, scope="CifarNet",
                 compat_double_softmax=False):
        super().__init__(scope)
        cinit = ("truncated_normal", 5e-2)
        self.conv1 = Conv2d(_join(scope, "conv1"), 3, 64, 5, 1, "SAME", "relu", None, True, 0.0, cinit)
        self.conv2 = Conv2d(_join(scope, "conv2"), 64, 64, 5, 1, "SAME", "relu", None, True, 0.0, cinit)
        self.fc3 = FullyConnected(_join(scope, "fc3"), 8 * 8 * 64, 384, "relu", None, True, weight_decay,
                                  ("truncated_normal", 0.04), 0.1)
        self.dropout3 = Dropout(_join(scope, "dropout3"), dropout_keep_prob)
        self.fc4 = FullyConnected(_join(scope, "fc4"), 384, 192, "relu", None, True, weight_decay,
                                  ("truncated_normal", 0.04), 0.1)
        self.logits = FullyConnected(_join(scope, "logits"), 192, num_classes, None, None, True, 0.0,
                                     ("truncated_normal", 1 / 192.0), 0.0)
        self.compat_double_softmax = compat_double_softmax

    def forward(self, x, training=True, end_points=None):
        net = F.max_pool(self.conv1(x, training), 2, 2, "VALID")
        net = lrn(net, 4, 1.0, 0.001 / 9.0, 0.75)
        net = self.conv2(net, training)
        net = lrn(net, 4, 1.0, 0.001 / 9.0, 0.75)
        net = F.max_pool(net, 2, 2, "VALID")
        net = self.fc3(_flatten(net), training)
        net = self.dropout3(net, training)
        net = self.fc4(net, training)
        logits = self.logits(net, training)
        if self.compat_double_softmax:  # cifarnet/cifarnet.py:94-95 returns Predictions
            return torch.softmax(logits.float(), -1)
        return logits


def _conv_fc(scope, cin, cout, k, padding, act, wd, init, bias_init):
    return Conv2d(scope, cin, cout, k, 1, padding, act, None, True, wd, init, bias_init)


class AlexNetV2(Layer):
    default_image_size = 224

    def __init__(self, num_classes=1000, dropout_keep_prob=0.5, spatial_squeeze=True, scope="alexnet_v2",
                 weight_decay=0.0, global_pool=False, arg_scope=False, cifar_variant=None):
        """arg_scope=False reproduces the reference call (no alexnet_v2_arg_scope: slim defaults,
        max_pool2d VALID, biases 0); True applies the reference's alexnet_v2_arg_scope (biases 0.1,
        pools SAME, alexnet/alexnet.py:45-53).  cifar_variant (default: num_classes == 10) selects
        the reference's patched geometry (stride-1 conv1, 5x5 'SAME' fc6); otherwise the upstream
        224 geometry (stride-4 conv1, 'VALID' fc6) so logits squeeze to [B, classes]."""
        super().__init__(scope)
        if cifar_variant is None:
            cifar_variant = num_classes == 10
        self.pool_pad = "SAME" if arg_scope else "VALID"
        fc6_pad = "SAME" if cifar_variant else "VALID"
        b0 = 0.1 if arg_scope else 0.0
        wd = weight_decay
        s1 = 1 if cifar_variant else 4  # CIFAR branch (alexnet/alexnet.py:102-105)
        self.conv1 = Conv2d(_join(scope, "conv1"), 3, 64, 11, s1, "VALID", "relu", None, True, wd, "xavier", b0)
        self.conv2 = Conv2d(_join(scope, "conv2"), 64, 192, 5, 1, "SAME", "relu", None, True, wd, "xavier", b0)
        self.conv3 = Conv2d(_join(scope, "conv3"), 192, 384, 3, 1, "SAME", "relu", None, True, wd, "xavier", b0)
        self.conv4 = Conv2d(_join(scope, "conv4"), 384, 384, 3, 1, "SAME", "relu", None, True, wd, "xavier", b0)
        self.conv5 = Conv2d(_join(scope, "conv5"), 384, 256, 3, 1, "SAME", "relu", None, True, wd, "xavier", b0)
        tn = ("truncated_normal", 0.005)
        self.fc6 = _conv_fc(_join(scope, "fc6"), 256, 4096, 5, fc6_pad, "relu", wd, tn, 0.1)
        self.dropout6 = Dropout(_join(scope, "dropout6"), dropout_keep_prob)
        self.fc7 = _conv_fc(_join(scope, "fc7"), 4096, 4096, 1, "SAME", "relu", wd, tn, 0.1)
        self.dropout7 = Dropout(_join(scope, "dropout7"), dropout_keep_prob)
        self.fc8 = _conv_fc(_join(scope, "fc8"), 4096, num_classes, 1, "SAME", None, wd, tn, 0.0) \
            if num_classes else None
        self.spatial_squeeze, self.global_pool = spatial_squeeze, global_pool

    def forward(self, x, training=True, end_points=None):
        net = F.max_pool(self.conv1(x, training), 3, 2, self.pool_pad)
        net = F.max_pool(self.conv2(net, training), 3, 2, self.pool_pad)
        net = self.conv5(self.conv4(self.conv3(net, training), training), training)
        net = F.max_pool(net, 3, 2, self.pool_pad)
        net = self.dropout6(self.fc6(net, training), training)
        net = self.fc7(net, training)
        if self.global_pool:
            net = F.global_avg_pool(net).reshape(net.shape[0], 1, 1, -1)
        if self.fc8 is None:
            return net
        net = self.fc8(self.dropout7(net, training), training)
        if self.spatial_squeeze:
            if net.shape[1] != 1 or net.shape[2] != 1:
                raise ValueError("cannot squeeze spatial dims %s (use a %dx%d input or global_pool=True)" % (
                    tuple(net.shape), self.default_image_size, self.default_image_size))
            net = net.reshape(net.shape[0], -1)
        return net


VGG_CFG = {"vgg_a": [1, 1, 2, 2, 2], "vgg_16": [2, 2, 3, 3, 3], "vgg_19": [2, 2, 4, 4, 4]}


class VGG(Layer):
    default_image_size = 224

    def __init__(self, variant="vgg_16", num_classes=1000, dropout_keep_prob=0.5, spatial_squeeze=True, scope=None,
                 fc_conv_padding="VALID", weight_decay=0.0005, global_pool=False):
        scope = scope or variant
        super().__init__(scope)
        widths = [64, 128, 256, 512, 512]
        convs = []
        cin = 3
        self.blocks = []
        for bi, (n, w) in enumerate(zip(VGG_CFG[variant], widths)):
            blk = []
            for i in range(n):
                name = _join(scope, "conv%d/conv%d_%d" % (bi + 1, bi + 1, i + 1))
                c = Conv2d(name, cin, w, 3, 1, "SAME", "relu", None, True, weight_decay, "xavier", 0.0)
                convs.append(c)
                blk.append(c)
                cin = w
            self.blocks.append(blk)
        self.convs = torch.nn.ModuleList(convs)
        self.fc6 = Conv2d(_join(scope, "fc6"), 512, 4096, 7, 1, fc_conv_padding, "relu", None, True, weight_decay,
                          "xavier", 0.0)
        self.dropout6 = Dropout(_join(scope, "dropout6"), dropout_keep_prob)
        self.fc7 = Conv2d(_join(scope, "fc7"), 4096, 4096, 1, 1, "SAME", "relu", None, True, weight_decay, "xavier", 0.0)
        self.dropout7 = Dropout(_join(scope, "dropout7"), dropout_keep_prob)
        self.fc8 = Conv2d(_join(scope, "fc8"), 4096, num_classes, 1, 1, "SAME", None, None, True, weight_decay,
                          "xavier", 0.0) if num_classes else None
        self.spatial_squeeze, self.global_pool = spatial_squeeze, global_pool

    def forward(self, x, training=True, end_points=None):
        net = x
        for bi, blk in enumerate(self.blocks):
            for c in blk:
                net = c(net, training)
            net = F.max_pool(net, 2, 2, "VALID")
            if end_points is not None:
                end_points[_join(self.scope, "pool%d" % (bi + 1))] = net
        net = self.dropout6(self.fc6(net, training), training)
        net = self.fc7(net, training)
        if self.global_pool:
            net = F.global_avg_pool(net).reshape(net.shape[0], 1, 1, -1)
        if self.fc8 is None:
            return net
        net = self.fc8(self.dropout7(net, training), training)
        if self.spatial_squeeze:
            net = net.reshape(net.shape[0], -1) if net.shape[1] == 1 and net.shape[2] == 1 else \
                _raise_squeeze(net)
        return net


def _raise_squeeze(net):
    raise ValueError("cannot squeeze spatial dims of %s (fc_conv_padding='same' at 224 keeps a 7x7 map; "
                     "the reference vgg copy has the same defect, SURVEY.md §4.2)" % (tuple(net.shape),))


class OverFeat(Layer):
    default_image_size = 231

    def __init__(self, num_classes=1000, dropout_keep_prob=0.5, spatial_squeeze=True, scope="overfeat",
                 weight_decay=0.0005, global_pool=False):
        super().__init__(scope)
        wd = weight_decay
        self.conv1 = Conv2d(_join(scope, "conv1"), 3, 64, 11, 4, "VALID", "relu", None, True, wd, "xavier", 0.1)
        self.conv2 = Conv2d(_join(scope, "conv2"), 64, 256, 5, 1, "VALID", "relu", None, True, wd, "xavier", 0.1)
        self.conv3 = Conv2d(_join(scope, "conv3"), 256, 512, 3, 1, "SAME", "relu", None, True, wd, "xavier", 0.1)
        self.conv4 = Conv2d(_join(scope, "conv4"), 512, 1024, 3, 1, "SAME", "relu", None, True, wd, "xavier", 0.1)
        self.conv5 = Conv2d(_join(scope, "conv5"), 1024, 1024, 3, 1, "SAME", "relu", None, True, wd, "xavier", 0.1)
        tn = ("truncated_normal", 0.005)
        self.fc6 = _conv_fc(_join(scope, "fc6"), 1024, 3072, 6, "VALID", "relu", wd, tn, 0.1)
        self.dropout6 = Dropout(_join(scope, "dropout6"), dropout_keep_prob)
        self.fc7 = _conv_fc(_join(scope, "fc7"), 3072, 4096, 1, "SAME", "relu", wd, tn, 0.1)
        self.dropout7 = Dropout(_join(scope, "dropout7"), dropout_keep_prob)
        self.fc8 = _conv_fc(_join(scope, "fc8"), 4096, num_classes, 1, "SAME", None, wd, tn, 0.0) \
            if num_classes else None
        self.spatial_squeeze, self.global_pool = spatial_squeeze, global_pool

    def forward(self, x, training=True, end_points=None):
        net = F.max_pool(self.conv1(x, training), 2, 2, "VALID")
        net = F.max_pool(self.conv2(net, training), 2, 2, "VALID")
        net = self.conv5(self.conv4(self.conv3(net, training), training), training)
        net = F.max_pool(net, 2, 2, "VALID")
        net = self.dropout6(self.fc6(net, training), training)
        net = self.fc7(net, training)
        if self.global_pool:
            net = F.global_avg_pool(net).reshape(net.shape[0], 1, 1, -1)
        if self.fc8 is None:
            return net
        net = self.fc8(self.dropout7(net, training), training)
        if self.spatial_squeeze:
            net = net.reshape(net.shape[0], -1)
        return net
