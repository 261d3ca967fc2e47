"""ResNet v2 in the official-models style (reference resnet/resnet_model.py:41-370), used by the
``resnet`` CIFAR trainer (cifar10_resnet_v2_generator, 6n+2 layers, filters 16/32/64) and
``imagenet_resnet_v2`` (18..200).

Pre-activation units (BN -> ReLU -> conv); projection shortcut taken from the *activated*
input; ``conv2d_fixed_padding`` (explicit symmetric pad + VALID when strided); BN decay 0.997,
eps 1e-5, center+scale; variance-scaling init; no conv biases; final BN-ReLU, average pool,
dense.  Variable names follow tf.layers auto-naming in creation order under the trainer's
'root' scope: root/conv2d{,_1..}/kernel, root/batch_normalization{,_1..}/{gamma,beta,moving_*},
root/dense/{kernel,bias}  (SURVEY.md §5.4).
"""
import torch

from ..ops import nn as F
from .layers import BatchNorm, Conv2d, FullyConnected, Layer

_BN = dict(decay=0.997, epsilon=1e-5, scale=True, bessel=True)


class _Namer:
    def __init__(self, scope):
        self.scope = scope + "/" if scope else ""
        self.c = {}

    def __call__(self, base):
        n = self.c.get(base, 0)
        self.c[base] = n + 1
        return self.scope + (base if n == 0 else "%s_%d" % (base, n))


def _rename(layer, mapping):
    for p_name, new in mapping.items():
        p = getattr(layer, p_name, None)
        if p is not None:
            p.tf_name = new


class _Conv(Conv2d):
    """tf.layers.conv2d: <name>/kernel (HWIO), no bias."""

    def __init__(self, name, cin, cout, k, stride, wd):
        pad = "SAME" if stride == 1 else ((k - 1) // 2, (k - 1) // 2)
        super().__init__(name, cin, cout, k, stride, pad, None, None, False, wd, "variance_scaling")
        self.weights.tf_name = name + "/kernel"


class _BNLayer(BatchNorm):
    def __init__(self, name, c):
        super().__init__(name, c, **_BN)


class _Block(Layer):
    def __init__(self, nm, cin, filters, stride, bottleneck, projection, wd):
        super().__init__("")
        out = filters * 4 if bottleneck else filters
        self.bn1 = _BNLayer(nm("batch_normalization"), cin)
        self.proj = _Conv(nm("conv2d"), cin, out, 1, stride, wd) if projection else None
        if bottleneck:
            self.c1 = _Conv(nm("conv2d"), cin, filters, 1, 1, wd)
            self.bn2 = _BNLayer(nm("batch_normalization"), filters)
            self.c2 = _Conv(nm("conv2d"), filters, filters, 3, stride, wd)
            self.bn3 = _BNLayer(nm("batch_normalization"), filters)
            self.c3 = _Conv(nm("conv2d"), filters, out, 1, 1, wd)
        else:
            self.c1 = _Conv(nm("conv2d"), cin, filters, 3, stride, wd)
            self.bn2 = _BNLayer(nm("batch_normalization"), filters)
            self.c2 = _Conv(nm("conv2d"), filters, filters, 3, 1, wd)
        self.bottleneck = bottleneck

    def forward(self, x, training=True):
        shortcut = x
        a = self.bn1(x, training, relu=True)
        if self.proj is not None:
            shortcut = self.proj(a, training)
        y = self.bn2(self.c1(a, training), training, relu=True)
        y = self.c2(y, training)
        if self.bottleneck:
            y = self.c3(self.bn3(y, training, relu=True), training)
        from ..ops.lazy import as_tensor
        return as_tensor(y) + as_tensor(shortcut).to(as_tensor(y).dtype)


class CifarResNetV2(Layer):
    """cifar10_resnet_v2_generator(resnet_size, num_classes): resnet_size = 6n + 2."""
    default_image_size = 32

    def __init__(self, resnet_size=32, num_classes=10, scope="root", weight_decay=0.0):
        super().__init__(scope)
        if resnet_size % 6 != 2:
            raise ValueError("resnet_size must be 6n + 2:", resnet_size)
        n = (resnet_size - 2) // 6
        nm = _Namer(scope)
        self.initial = _Conv(nm("conv2d"), 3, 16, 3, 1, weight_decay)
        blocks, cin = [], 16
        for filters, stride in ((16, 1), (32, 2), (64, 2)):
            for i in range(n):
                blocks.append(_Block(nm, cin, filters, stride if i == 0 else 1, False, i == 0,
                                    weight_decay))
                cin = filters
        self.blocks = torch.nn.ModuleList(blocks)
        self.final_bn = _BNLayer(nm("batch_normalization"), 64)
        self.dense = FullyConnected(nm("dense"), 64, num_classes, None, None, True, weight_decay, "xavier")
        _rename(self.dense, {"weights": self.dense.scope + "/kernel", "biases": self.dense.scope + "/bias"})

    def forward(self, x, training=True, end_points=None):
        net = self.initial(x, training)
        for b in self.blocks:
            net = b(net, training)
        net = self.final_bn(net, training, relu=True)
        net = F.global_avg_pool(net)  # 8x8 average pool on 32x32 inputs
        return self.dense(net, training)


IMAGENET_CFG = {18: ("basic", [2, 2, 2, 2]), 34: ("basic", [3, 4, 6, 3]), 50: ("bottleneck", [3, 4, 6, 3]),
                101: ("bottleneck", [3, 4, 23, 3]), 152: ("bottleneck", [3, 8, 36, 3]),
                200: ("bottleneck", [3, 24, 36, 3])}


class ImagenetResNetV2(Layer):
    """imagenet_resnet_v2(resnet_size, num_classes) (resnet/resnet_model.py:285-370)."""
    default_image_size = 224

    def __init__(self, resnet_size=50, num_classes=1001, scope="", weight_decay=0.0):
        super().__init__(scope)
        kind, layers = IMAGENET_CFG[resnet_size]
        bott = kind == "bottleneck"
        nm = _Namer(scope)
        self.initial = _Conv(nm("conv2d"), 3, 64, 7, 2, weight_decay)
        blocks, cin = [], 64
        for li, (filters, stride) in enumerate(((64, 1), (128, 2), (256, 2), (512, 2))):
            out = filters * 4 if bott else filters
            for i in range(layers[li]):
                blocks.append(_Block(nm, cin, filters, stride if i == 0 else 1, bott, i == 0,
                                     weight_decay))
                cin = out
        self.blocks = torch.nn.ModuleList(blocks)
        self.final_bn = _BNLayer(nm("batch_normalization"), cin)
        self.dense = FullyConnected(nm("dense"), cin, num_classes, None, None, True, weight_decay, "xavier")
        _rename(self.dense, {"weights": self.dense.scope + "/kernel", "biases": self.dense.scope + "/bias"})

    def forward(self, x, training=True, end_points=None):
        net = self.initial(x, training)
        net = F.max_pool(net, 3, 2, "SAME")
        for b in self.blocks:
            net = b(net, training)
        net = self.final_bn(net, training, relu=True)
        net = F.global_avg_pool(net)
        return self.dense(net, training)
