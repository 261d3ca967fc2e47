"""Model registry (reference vgg/nets/nets_factory.py:39-145: networks_map / get_network_fn).

``build(name, num_classes)`` returns an nn.Module taking NHWC images; ``get_network_fn`` mirrors
slim's factory (returns fn(images) -> (logits, end_points) with ``default_image_size``).
The names include everything in the reference registry plus the reference's own trainer models
(cifar10 CNN, CIFAR ResNet v2, old-slim Inception-v3).
"""
import functools

from . import classic, resnet_official, resnet_v1, slim_nets
from .inception_v3_slim import InceptionV3Slim
from .slim_model import SlimModel


def _slim(fn, size, **defaults):
    def make(num_classes=1000, **kw):
        d = dict(defaults)
        d.update(kw)
        return SlimModel(fn, size, num_classes=num_classes, name=fn.__name__, **d)
    make.default_image_size = size
    return make


def _lazy(modname, attr, size, **defaults):
    """Models living in optional modules (NASNet, GANs) are imported on first use."""
    def make(num_classes=1000, **kw):
        import importlib
        mod = importlib.import_module("distributed_tensorflow_models_amd.models." + modname)
        d = dict(defaults)
        d.update(kw)
        return SlimModel(getattr(mod, attr), size, num_classes=num_classes, name=attr, **d)
    make.default_image_size = size
    return make


networks_map = {
    # classic
    "cifar10_cnn": lambda num_classes=10, **kw: classic.Cifar10CNN(num_classes, **kw),
    "lenet": lambda num_classes=10, **kw: classic.LeNet(num_classes, **kw),
    "cifarnet": lambda num_classes=10, **kw: classic.CifarNet(num_classes, **kw),
    "alexnet_v2": lambda num_classes=1000, **kw: classic.AlexNetV2(num_classes, **kw),
    "overfeat": lambda num_classes=1000, **kw: classic.OverFeat(num_classes, **kw),
    "vgg_a": lambda num_classes=1000, **kw: classic.VGG("vgg_a", num_classes, **kw),
    "vgg_16": lambda num_classes=1000, **kw: classic.VGG("vgg_16", num_classes, **kw),
    "vgg_19": lambda num_classes=1000, **kw: classic.VGG("vgg_19", num_classes, **kw),
    # resnets
    "resnet_v1_50": resnet_v1.resnet_v1_50,
    "resnet_v1_101": resnet_v1.resnet_v1_101,
    "resnet_v1_152": resnet_v1.resnet_v1_152,
    "resnet_v1_200": resnet_v1.resnet_v1_200,
    "resnet_v2_50": _slim(slim_nets.resnet_v2, 224, depth=50),
    "resnet_v2_101": _slim(slim_nets.resnet_v2, 224, depth=101),
    "resnet_v2_152": _slim(slim_nets.resnet_v2, 224, depth=152),
    "resnet_v2_200": _slim(slim_nets.resnet_v2, 224, depth=200),
    "cifar10_resnet_v2": lambda num_classes=10, resnet_size=32, **kw: resnet_official.CifarResNetV2(
        resnet_size, num_classes, **kw),
    "imagenet_resnet_v2": lambda num_classes=1001, resnet_size=50, **kw: resnet_official.ImagenetResNetV2(
        resnet_size, num_classes, **kw),
    # inception family
    "inception_v1": _slim(slim_nets.inception_v1, 224),
    "inception_v2": _slim(slim_nets.inception_v2, 224),
    "inception_v3": _slim(slim_nets.inception_v3, 299),
    "inception_v3_slim_old": lambda num_classes=1001, **kw: InceptionV3Slim(num_classes, **kw),
    "inception_v4": _lazy("inception_v4", "inception_v4", 299),
    "inception_resnet_v2": _lazy("inception_v4", "inception_resnet_v2", 299),
    # mobile
    "mobilenet_v1": _slim(slim_nets.mobilenet_v1, 224),
    "mobilenet_v1_075": _slim(slim_nets.mobilenet_v1, 224, depth_multiplier=0.75),
    "mobilenet_v1_050": _slim(slim_nets.mobilenet_v1, 160, depth_multiplier=0.50),
    "mobilenet_v1_025": _slim(slim_nets.mobilenet_v1, 128, depth_multiplier=0.25),
    "mobilenet_v2": _slim(slim_nets.mobilenet_v2, 224),
    "mobilenet_v2_140": _slim(slim_nets.mobilenet_v2, 224, depth_multiplier=1.4),
    "mobilenet_v2_035": _slim(slim_nets.mobilenet_v2, 224, depth_multiplier=0.35),
    "nasnet_cifar": _lazy("nasnet", "build_nasnet_cifar", 32),
    "nasnet_mobile": _lazy("nasnet", "build_nasnet_mobile", 224),
    "nasnet_large": _lazy("nasnet", "build_nasnet_large", 331),
    "pnasnet_large": _lazy("nasnet", "build_pnasnet_large", 331),
}


def build(name, num_classes=1000, **kw):
    if name not in networks_map:
        raise ValueError("Name of network unknown %s" % name)
    return networks_map[name](num_classes=num_classes, **kw)


def default_image_size(name):
    fn = networks_map[name]
    s = getattr(fn, "default_image_size", None)
    if s is None:
        s = getattr(build(name, 10), "default_image_size", 224)
    return s


def get_network_fn(name, num_classes, weight_decay=0.0, is_training=False, **kw):
    """fn(images) -> (logits, end_points) like slim's nets_factory.get_network_fn."""
    net = build(name, num_classes, **kw)

    @functools.wraps(net.forward)
    def network_fn(images, **call_kw):
        ep = {}
        logits = net(images, training=call_kw.get("training", is_training), end_points=ep)
        return logits, ep

    network_fn.default_image_size = getattr(net, "default_image_size", 224)
    network_fn.module = net
    return network_fn
