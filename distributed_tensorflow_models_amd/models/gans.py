"""GAN model zoo: DCGAN generator/discriminator, CycleGAN ResNet generator, pix2pix U-Net
generator and PatchGAN discriminator (reference vgg/nets/dcgan.py:24-202,
vgg/nets/cyclegan.py:29-273, vgg/nets/pix2pix.py:25-292), on the functional slim facade.

Transposed convolutions run on the HIP implicit-GEMM dgrad kernel (ops.nn.conv2d_transpose);
instance normalisation, reflect padding and nearest-neighbour upsampling are plain tensor ops.
"""
import math

import torch

from ..compat import slim
from ..ops.lazy import as_tensor


def _lrelu(x):
    return slim.leaky_relu(x, 0.2)


def _is_pow2(n):
    return n > 0 and (n & (n - 1)) == 0


# ---------------------------------------------------------------------------------------------
# DCGAN (dcgan.py)
def dcgan_discriminator(inputs, depth=64, is_training=True, scope="Discriminator", fused_batch_norm=False):
    x = as_tensor(inputs)
    if x.dim() != 4 or x.shape[1] != x.shape[2] or not _is_pow2(int(x.shape[1])):
        raise ValueError("Input must be square with a power-of-2 size, got %s" % (tuple(x.shape),))
    ep = {}
    with slim.variable_scope(scope):
        with slim.arg_scope([slim.batch_norm], is_training=is_training, scale=False), \
                slim.arg_scope([slim.conv2d], stride=2, kernel_size=4, activation_fn=_lrelu):
            net = x
            for i in range(int(math.log2(x.shape[1]))):
                name = "conv%d" % (i + 1)
                net = ep[name] = slim.conv2d(net, depth * 2 ** i, normalizer_fn=None if i == 0 else slim.batch_norm,
                                             scope=name)
            logits = slim.conv2d(net, 1, kernel_size=1, stride=1, padding="VALID", normalizer_fn=None,
                                 activation_fn=None)
            logits = ep["logits"] = as_tensor(logits).reshape(-1, 1)
    return logits, ep


def dcgan_generator(inputs, depth=64, final_size=32, num_outputs=3, is_training=True, scope="Generator",
                    fused_batch_norm=False):
    x = as_tensor(inputs)
    if x.dim() != 2:
        raise ValueError("generator inputs must be rank 2")
    if not _is_pow2(final_size):
        raise ValueError("`final_size` (%i) must be a power of 2." % final_size)
    if final_size < 8:
        raise ValueError("`final_size` (%i) must be greater than 8." % final_size)
    ep = {}
    n = int(math.log2(final_size)) - 1
    with slim.variable_scope(scope):
        with slim.arg_scope([slim.batch_norm], is_training=is_training, scale=False), \
                slim.arg_scope([slim.conv2d_transpose], normalizer_fn=slim.batch_norm, stride=2, kernel_size=4):
            net = x.reshape(x.shape[0], 1, 1, x.shape[1])
            net = ep["deconv1"] = slim.conv2d_transpose(net, depth * 2 ** (n - 1), stride=1, padding="VALID",
                                                        scope="deconv1")
            for i in range(2, n):
                net = ep["deconv%d" % i] = slim.conv2d_transpose(net, depth * 2 ** (n - i), scope="deconv%d" % i)
            net = ep["deconv%d" % n] = slim.conv2d_transpose(net, depth, normalizer_fn=None, activation_fn=None,
                                                             scope="deconv%d" % n)
            logits = ep["logits"] = slim.conv2d(net, num_outputs, normalizer_fn=None, activation_fn=None,
                                                kernel_size=1, stride=1, padding="VALID", scope="logits")
    assert tuple(logits.shape[1:]) == (final_size, final_size, num_outputs)
    return logits, ep


# ---------------------------------------------------------------------------------------------
# CycleGAN (cyclegan.py)
class _Ctx:
    def __init__(self, *cms):
        self.cms = cms

    def __enter__(self):
        for c in self.cms:
            c.__enter__()

    def __exit__(self, *a):
        for c in reversed(self.cms):
            c.__exit__(*a)


def cyclegan_arg_scope(instance_norm_center=True, instance_norm_scale=True, instance_norm_epsilon=0.001,
                       weights_init_stddev=0.02, weight_decay=0.0):
    reg = slim.l2_regularizer(weight_decay) if weight_decay and weight_decay > 0 else None
    return _Ctx(slim.arg_scope([slim.conv2d], normalizer_fn=slim.instance_norm,
                               normalizer_params=dict(center=instance_norm_center, scale=instance_norm_scale,
                                                      epsilon=instance_norm_epsilon),
                               weights_initializer=slim.random_normal_initializer(0, weights_init_stddev),
                               weights_regularizer=reg))


def _nn_resize(x, sh, sw):
    x = as_tensor(x)
    return x.repeat_interleave(sh, dim=1).repeat_interleave(sw, dim=2)


def cyclegan_upsample(net, num_outputs, stride, method="conv2d_transpose"):
    with slim.variable_scope("upconv"):
        if method == "nn_upsample_conv":
            net = slim.reflect_pad(_nn_resize(net, stride[0], stride[1]), 1, 1, 1, 1)
            return slim.conv2d(net, num_outputs, kernel_size=3, padding="VALID")
        if method == "bilinear_upsample_conv":
            x = as_tensor(net)
            x = torch.nn.functional.interpolate(x.permute(0, 3, 1, 2).float(), scale_factor=tuple(stride),
                                                mode="bilinear", align_corners=False).permute(0, 2, 3, 1).to(x.dtype)
            return slim.conv2d(slim.reflect_pad(x, 1, 1, 1, 1), num_outputs, kernel_size=3, padding="VALID")
        if method == "conv2d_transpose":
            net = slim.conv2d_transpose(net, num_outputs, kernel_size=3, stride=stride[0], padding="VALID")
            return as_tensor(net)[:, 1:, 1:, :]
        raise ValueError("Unknown method: [%s]" % method)


def cyclegan_generator_resnet(images, arg_scope_fn=cyclegan_arg_scope, num_resnet_blocks=6, num_filters=64,
                              upsample_fn=cyclegan_upsample, kernel_size=3, num_outputs=3, tanh_linear_slope=0.0,
                              is_training=False):
    x = as_tensor(images)
    H, W = x.shape[1], x.shape[2]
    if H % 4:
        raise ValueError("The input height must be a multiple of 4.")
    if W % 4:
        raise ValueError("The input width must be a multiple of 4.")
    kh, kw = (kernel_size, kernel_size) if isinstance(kernel_size, int) else kernel_size
    pads = ((kh - 1) // 2, kh // 2, (kw - 1) // 2, kw // 2)
    ep = {}
    with arg_scope_fn():
        with slim.variable_scope("input"):
            net = ep["encoder_0"] = slim.conv2d(slim.reflect_pad(x, 3, 3, 3, 3), num_filters, kernel_size=7,
                                                padding="VALID")
        with slim.variable_scope("encoder"), \
                slim.arg_scope([slim.conv2d], kernel_size=(kh, kw), stride=2, activation_fn=torch.relu,
                               padding="VALID"):
            net = ep["encoder_1"] = slim.conv2d(slim.reflect_pad(net, *pads), num_filters * 2)
            net = ep["encoder_2"] = slim.conv2d(slim.reflect_pad(net, *pads), num_filters * 4)
        with slim.variable_scope("residual_blocks"), \
                slim.arg_scope([slim.conv2d], kernel_size=(kh, kw), stride=1, activation_fn=torch.relu,
                               padding="VALID"):
            for b in range(num_resnet_blocks):
                with slim.variable_scope("block_%d" % b):
                    r = slim.conv2d(slim.reflect_pad(net, *pads), num_filters * 4)
                    r = slim.conv2d(slim.reflect_pad(r, *pads), num_filters * 4, activation_fn=None)
                    net = ep["resnet_block_%d" % b] = as_tensor(net) + as_tensor(r)
        with slim.variable_scope("decoder"), \
                slim.arg_scope([slim.conv2d], kernel_size=(kh, kw), stride=1, activation_fn=torch.relu):
            with slim.variable_scope("decoder1"):
                net = ep["decoder1"] = upsample_fn(net, num_outputs=num_filters * 2, stride=[2, 2])
            with slim.variable_scope("decoder2"):
                net = ep["decoder2"] = upsample_fn(net, num_outputs=num_filters, stride=[2, 2])
        with slim.variable_scope("output"):
            logits = slim.conv2d(slim.reflect_pad(net, 3, 3, 3, 3), num_outputs, 7, activation_fn=None,
                                 normalizer_fn=None, padding="VALID")
            logits = ep["logits"] = as_tensor(logits).reshape(x.shape[0], H, W, num_outputs)
            ep["predictions"] = torch.tanh(logits) + logits * tanh_linear_slope
    return ep["predictions"], ep


# ---------------------------------------------------------------------------------------------
# pix2pix (pix2pix.py)
def pix2pix_arg_scope():
    p = dict(center=True, scale=True, epsilon=1e-5)
    return _Ctx(slim.arg_scope([slim.conv2d, slim.conv2d_transpose], normalizer_fn=slim.instance_norm,
                               normalizer_params=p, weights_initializer=slim.random_normal_initializer(0, 0.02)))


def pix2pix_upsample(net, num_outputs, kernel_size, method="nn_upsample_conv"):
    if method == "nn_upsample_conv":
        return slim.conv2d(_nn_resize(net, kernel_size[0], kernel_size[1]), num_outputs, 4, activation_fn=None)
    if method == "conv2d_transpose":
        return slim.conv2d_transpose(net, num_outputs, 4, stride=kernel_size[0], activation_fn=None)
    raise ValueError("Unknown method: [%s]" % method)


PIX2PIX_BLOCKS = [(64, 0.5), (128, 0.5), (256, 0.5), (512, 0), (512, 0), (512, 0), (512, 0)]


def pix2pix_generator(net, num_outputs, blocks=None, upsample_method="nn_upsample_conv", is_training=False):
    x = as_tensor(net)
    if x.shape[1] != x.shape[2]:
        raise ValueError("The input height must match the input width.")
    blocks = blocks or PIX2PIX_BLOCKS
    ep = {}
    enc = []
    with slim.variable_scope("encoder"), \
            slim.arg_scope([slim.conv2d], kernel_size=4, stride=2, activation_fn=_lrelu):
        net = x
        for i, (nf, _keep) in enumerate(blocks):
            if i == 0:
                net = slim.conv2d(net, nf, normalizer_fn=None)
            elif i < len(blocks) - 1:
                net = slim.conv2d(net, nf)
            else:
                net = slim.conv2d(net, nf, activation_fn=None, normalizer_fn=None)
            enc.append(net)
            ep["encoder%d" % i] = net
    with slim.variable_scope("decoder"):
        for i, (nf, keep) in enumerate(reversed(blocks)):
            if i > 0:
                net = torch.cat([as_tensor(net), as_tensor(enc[-i - 1])], -1)
            net = pix2pix_upsample(torch.relu(as_tensor(net)), nf, [2, 2], upsample_method)
            if keep > 0:
                net = slim.dropout(net, keep_prob=keep, is_training=True)
            ep["decoder%d" % i] = net
    with slim.variable_scope("output"):
        logits = slim.conv2d(net, num_outputs, 4, activation_fn=None, normalizer_fn=None)
        logits = ep["logits"] = as_tensor(logits).reshape(x.shape[0], x.shape[1], x.shape[2], num_outputs)
        ep["predictions"] = torch.tanh(logits)
    return logits, ep


def pix2pix_discriminator(net, num_filters, padding=2, is_training=False):
    ep = {}
    n = len(num_filters)

    def padded(t, scope):
        if padding:
            with slim.variable_scope(scope):
                return slim.reflect_pad(t, padding, padding, padding, padding)
        return t

    with slim.arg_scope([slim.conv2d], kernel_size=4, stride=2, padding="VALID", activation_fn=_lrelu):
        net = ep["conv0"] = slim.conv2d(padded(net, "conv0"), num_filters[0], normalizer_fn=None, scope="conv0")
        for i in range(1, n - 1):
            net = ep["conv%d" % i] = slim.conv2d(padded(net, "conv%d" % i), num_filters[i], scope="conv%d" % i)
        net = ep["conv%d" % (n - 1)] = slim.conv2d(padded(net, "conv%d" % (n - 1)), num_filters[-1], stride=1,
                                                   scope="conv%d" % (n - 1))
        logits = ep["logits"] = slim.conv2d(padded(net, "conv%d" % n), 1, stride=1, activation_fn=None,
                                            normalizer_fn=None, scope="conv%d" % n)
        ep["predictions"] = torch.sigmoid(as_tensor(logits))
    return logits, ep
