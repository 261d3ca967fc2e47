"""Model registry (mirrors reference vgg/nets/nets_factory.py:39-145 networks_map/get_network_fn)."""
from . import resnet_v1

networks_map = {
    "resnet_v1_50": resnet_v1.resnet_v1_50,
    "resnet_v1_101": resnet_v1.resnet_v1_101,
    "resnet_v1_152": resnet_v1.resnet_v1_152,
    "resnet_v1_200": resnet_v1.resnet_v1_200,
}


def build(name, num_classes=1000, **kw):
    if name not in networks_map:
        raise ValueError("Name of network unknown %s" % name)
    return networks_map[name](num_classes=num_classes, **kw)


def get_network_fn(name, num_classes, weight_decay=0.0, is_training=False, **kw):
    """Returns fn(images) -> (logits, end_points) like slim's nets_factory."""
    net = build(name, num_classes, **kw)

    def network_fn(images, **call_kw):
        ep = {}
        logits = net(images, training=call_kw.get("training", is_training), end_points=ep)
        return logits, ep

    network_fn.default_image_size = getattr(net, "default_image_size", 224)
    network_fn.module = net
    return network_fn
