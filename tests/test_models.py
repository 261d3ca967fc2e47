"""Model-zoo structure goldens ported from the reference's TF tests: parameter
counts, TF variable names, endpoint shapes and output shapes, checked on CPU with the torch
oracle path (same model code as the HIP path)."""
import pytest
import torch

from distributed_tensorflow_models_amd.compat import slim
from distributed_tensorflow_models_amd.models import gans, inception_v4 as iv4, nasnet, nets_factory, slim_nets
from distributed_tensorflow_models_amd.models.layers import count_params, tf_variables
from distributed_tensorflow_models_amd.models.slim_model import SlimModel


def _run(fn, *a, **k):
    st = slim.VariableStore()
    with slim.use_store(st), torch.no_grad():
        slim.begin_pass()
        out = fn(*a, **k)
    return out, st


def _check_eps(ep, golden, exact_keys=True):
    got = {k: list(v.shape) for k, v in ep.items() if k in golden}
    assert got == golden
    if exact_keys:
        assert set(ep) == set(golden), sorted(set(ep) ^ set(golden))


# ---------------------------------------------------------------------------------------------
# parameter counts / variable layouts
@pytest.mark.parametrize("name,nc,total", [
    ("resnet_v1_50", 1000, 25557032),             # slim resnet_v1_50 (north-star model)
    ("inception_v3_slim_old", 1001, 27145970),    # inception/slim (collections_test layout)
    ("cifar10_resnet_v2", 10, 466970),            # resnet_size 32 (resnet/resnet_model.py)
])
def test_trainable_param_counts(name, nc, total):
    m = nets_factory.build(name, nc)
    assert sum(p.numel() for p in m.parameters() if p.requires_grad) == total


def test_vgg16_param_counts():
    assert count_params(nets_factory.build("vgg_16", 10, fc_conv_padding="SAME")) == 134301514
    assert count_params(nets_factory.build("vgg_16", 1000)) == 138357544


@pytest.mark.parametrize("fn,size,golden", [
    (slim_nets.inception_v1, 224, 5607184), (slim_nets.inception_v2, 224, 10173112),
    (slim_nets.inception_v3, 299, 21802784)])
def test_inception_base_model_variable_counts(fn, size, golden):
    # reference inception_v{1,2,3}_test.py testModelHasExpectedNumberOfParameters: all model
    # variables (incl. BN moving statistics) of the base network
    m = SlimModel(fn, size, num_classes=0)
    n = sum(p.numel() for p in m.parameters()) + sum(b.numel() for b in m.buffers())
    assert n == golden


def test_vgg16_variable_names():
    # reference vgg/nets/vgg_test.py:298-330 (testModelVariables, vgg_16)
    names = [n for n, *_ in tf_variables(nets_factory.build("vgg_16", 1000))]
    expected = []
    for blk, n in ((1, 2), (2, 2), (3, 3), (4, 3), (5, 3)):
        for i in range(1, n + 1):
            expected += ["vgg_16/conv%d/conv%d_%d/weights" % (blk, blk, i), "vgg_16/conv%d/conv%d_%d/biases" % (blk, blk, i)]
    for fc in ("fc6", "fc7", "fc8"):
        expected += ["vgg_16/%s/weights" % fc, "vgg_16/%s/biases" % fc]
    assert sorted(names) == sorted(expected)


def test_inception_resnet_v2_repeat_scopes():
    names = [n for n, *_ in tf_variables(nets_factory.build("inception_resnet_v2", 1001))]
    assert "InceptionResnetV2/Repeat/block35_10/Conv2d_1x1/weights" in names
    assert "InceptionResnetV2/Repeat_1/block17_20/Branch_1/Conv2d_0c_7x1/weights" in names
    assert "InceptionResnetV2/Repeat_2/block8_9/Conv2d_1x1/biases" in names
    assert "InceptionResnetV2/Block8/Conv2d_1x1/weights" in names
    assert "InceptionResnetV2/AuxLogits/Logits/weights" in names


# ---------------------------------------------------------------------------------------------
# endpoint shapes (reference *_test.py testBuildAndCheckAllEndPoints...)
def test_inception_v1_v2_v3_endpoints():
    B = 1
    ep = {}
    SlimModel(slim_nets.inception_v1, 224, num_classes=0)(torch.zeros(B, 224, 224, 3), training=False, end_points=ep)
    _check_eps(ep, {'Conv2d_1a_7x7': [B, 112, 112, 64], 'MaxPool_2a_3x3': [B, 56, 56, 64],
                    'Conv2d_2b_1x1': [B, 56, 56, 64], 'Conv2d_2c_3x3': [B, 56, 56, 192],
                    'MaxPool_3a_3x3': [B, 28, 28, 192], 'Mixed_3b': [B, 28, 28, 256], 'Mixed_3c': [B, 28, 28, 480],
                    'MaxPool_4a_3x3': [B, 14, 14, 480], 'Mixed_4b': [B, 14, 14, 512], 'Mixed_4c': [B, 14, 14, 512],
                    'Mixed_4d': [B, 14, 14, 512], 'Mixed_4e': [B, 14, 14, 528], 'Mixed_4f': [B, 14, 14, 832],
                    'MaxPool_5a_2x2': [B, 7, 7, 832], 'Mixed_5b': [B, 7, 7, 832], 'Mixed_5c': [B, 7, 7, 1024]},
               exact_keys=False)
    ep = {}
    SlimModel(slim_nets.inception_v2, 224, num_classes=0)(torch.zeros(B, 224, 224, 3), training=False, end_points=ep)
    _check_eps(ep, {'Mixed_3b': [B, 28, 28, 256], 'Mixed_3c': [B, 28, 28, 320], 'Mixed_4a': [B, 14, 14, 576],
                    'Mixed_4b': [B, 14, 14, 576], 'Mixed_4c': [B, 14, 14, 576], 'Mixed_4d': [B, 14, 14, 576],
                    'Mixed_4e': [B, 14, 14, 576], 'Mixed_5a': [B, 7, 7, 1024], 'Mixed_5b': [B, 7, 7, 1024],
                    'Mixed_5c': [B, 7, 7, 1024], 'Conv2d_1a_7x7': [B, 112, 112, 64],
                    'MaxPool_2a_3x3': [B, 56, 56, 64], 'Conv2d_2b_1x1': [B, 56, 56, 64],
                    'Conv2d_2c_3x3': [B, 56, 56, 192], 'MaxPool_3a_3x3': [B, 28, 28, 192]}, exact_keys=False)
    ep = {}
    SlimModel(slim_nets.inception_v3, 299, num_classes=0)(torch.zeros(B, 299, 299, 3), training=False, end_points=ep)
    _check_eps(ep, {'Conv2d_1a_3x3': [B, 149, 149, 32], 'Conv2d_2a_3x3': [B, 147, 147, 32],
                    'Conv2d_2b_3x3': [B, 147, 147, 64], 'MaxPool_3a_3x3': [B, 73, 73, 64],
                    'Conv2d_3b_1x1': [B, 73, 73, 80], 'Conv2d_4a_3x3': [B, 71, 71, 192],
                    'MaxPool_5a_3x3': [B, 35, 35, 192], 'Mixed_5b': [B, 35, 35, 256], 'Mixed_5c': [B, 35, 35, 288],
                    'Mixed_5d': [B, 35, 35, 288], 'Mixed_6a': [B, 17, 17, 768], 'Mixed_6b': [B, 17, 17, 768],
                    'Mixed_6c': [B, 17, 17, 768], 'Mixed_6d': [B, 17, 17, 768], 'Mixed_6e': [B, 17, 17, 768],
                    'Mixed_7a': [B, 8, 8, 1280], 'Mixed_7b': [B, 8, 8, 2048], 'Mixed_7c': [B, 8, 8, 2048]},
               exact_keys=False)


def test_inception_v4_endpoints():
    B, nc = 2, 1000
    ep = {}
    m = nets_factory.build("inception_v4", nc)
    (logits, aux) = m(torch.zeros(B, 299, 299, 3), training=True, end_points=ep)
    g = {'Conv2d_1a_3x3': [B, 149, 149, 32], 'Conv2d_2a_3x3': [B, 147, 147, 32], 'Conv2d_2b_3x3': [B, 147, 147, 64],
         'Mixed_3a': [B, 73, 73, 160], 'Mixed_4a': [B, 71, 71, 192], 'Mixed_5a': [B, 35, 35, 384]}
    g.update({'Mixed_5' + c: [B, 35, 35, 384] for c in "bcde"})
    g['Mixed_6a'] = [B, 17, 17, 1024]
    g.update({'Mixed_6' + c: [B, 17, 17, 1024] for c in "bcdefgh"})
    g['Mixed_7a'] = [B, 8, 8, 1536]
    g.update({'Mixed_7' + c: [B, 8, 8, 1536] for c in "bcd"})
    g.update({'AuxLogits': [B, nc], 'global_pool': [B, 1, 1, 1536], 'PreLogitsFlatten': [B, 1536],
              'Logits': [B, nc], 'Predictions': [B, nc]})
    _check_eps(ep, g)
    assert list(aux.shape) == [B, nc]


@pytest.mark.parametrize("kw,golden", [
    ({}, {'Conv2d_1a_3x3': [149, 32], 'Conv2d_2a_3x3': [147, 32], 'Conv2d_2b_3x3': [147, 64],
          'MaxPool_3a_3x3': [73, 64], 'Conv2d_3b_1x1': [73, 80], 'Conv2d_4a_3x3': [71, 192],
          'MaxPool_5a_3x3': [35, 192], 'Mixed_5b': [35, 320], 'Mixed_6a': [17, 1088], 'PreAuxLogits': [17, 1088]}),
    ({"align_feature_maps": True},
     {'Conv2d_1a_3x3': [150, 32], 'Conv2d_2a_3x3': [150, 32], 'Conv2d_2b_3x3': [150, 64],
      'MaxPool_3a_3x3': [75, 64], 'Conv2d_3b_1x1': [75, 80], 'Conv2d_4a_3x3': [75, 192],
      'MaxPool_5a_3x3': [38, 192], 'Mixed_5b': [38, 320], 'Mixed_6a': [19, 1088], 'PreAuxLogits': [19, 1088]}),
    ({"output_stride": 8},
     {'Conv2d_1a_3x3': [149, 32], 'Conv2d_2a_3x3': [147, 32], 'Conv2d_2b_3x3': [147, 64],
      'MaxPool_3a_3x3': [73, 64], 'Conv2d_3b_1x1': [73, 80], 'Conv2d_4a_3x3': [71, 192],
      'MaxPool_5a_3x3': [35, 192], 'Mixed_5b': [35, 320], 'Mixed_6a': [33, 1088], 'PreAuxLogits': [33, 1088]}),
])
def test_inception_resnet_v2_base_endpoints(kw, golden):
    B = 1
    ep = {}

    def fn(x):
        with slim.arg_scope([slim.batch_norm], is_training=False), \
                slim.arg_scope([slim.conv2d], normalizer_fn=slim.batch_norm):
            return iv4.inception_resnet_v2_base(x, ep, final_endpoint="PreAuxLogits", **kw)
    _run(fn, torch.zeros(B, 299, 299, 3))
    _check_eps(ep, {k: [B, s, s, c] for k, (s, c) in golden.items()})


def test_mobilenet_v1_endpoints():
    B = 1
    ep = {}
    nets_factory.build("mobilenet_v1", 1000)(torch.zeros(B, 224, 224, 3), training=False, end_points=ep)
    g = {'Conv2d_0': [B, 112, 112, 32]}
    dims = [(112, 32, 64), (56, 64, 128), (56, 128, 128), (28, 128, 256), (28, 256, 256), (14, 256, 512)] + \
        [(14, 512, 512)] * 5 + [(7, 512, 1024), (7, 1024, 1024)]
    for i, (s, cd, cp) in enumerate(dims, 1):
        g['Conv2d_%d_depthwise' % i] = [B, s, s, cd]
        g['Conv2d_%d_pointwise' % i] = [B, s, s, cp]
    _check_eps(ep, g, exact_keys=False)


@pytest.mark.parametrize("name,size,nc,golden", [
    ("nasnet_cifar", 32, 10, dict(Stem=[32, 96], **{"Cell_%d" % i: [32 if i < 6 else 16 if i < 12 else 8,
                                                                  192 if i < 6 else 384 if i < 12 else 768]
                                                    for i in range(18)},
                                  Reduction_Cell_0=[16, 256], Reduction_Cell_1=[8, 512])),
    ("nasnet_mobile", 224, 1000, dict(Stem=[28, 88], **{"Cell_%d" % i: [28 if i < 4 else 14 if i < 8 else 7,
                                                                       264 if i < 4 else 528 if i < 8 else 1056]
                                                         for i in range(12)},
                                      Reduction_Cell_0=[14, 352], Reduction_Cell_1=[7, 704])),
])
def test_nasnet_endpoints(name, size, nc, golden):
    B = 2
    ep = {}
    m = nets_factory.build(name, nc)
    out = m(torch.zeros(B, size, size, 3), training=True, end_points=ep)
    want = {k: [B, s, s, c] for k, (s, c) in golden.items()}
    pool = golden["Cell_%d" % (len([k for k in golden if k.startswith("Cell_")]) - 1)][1]
    want.update(global_pool=[B, pool], AuxLogits=[B, nc], Logits=[B, nc], Predictions=[B, nc])
    _check_eps(ep, want)
    assert isinstance(out, tuple) and list(out[0].shape) == [B, nc]


@pytest.mark.slow
@pytest.mark.parametrize("name,golden", [
    ("nasnet_large", dict(Stem=[42, 336], **{"Cell_%d" % i: [42 if i < 6 else 21 if i < 12 else 11,
                                                              1008 if i < 6 else 2016 if i < 12 else 4032]
                                              for i in range(18)},
                          Reduction_Cell_0=[21, 1344], Reduction_Cell_1=[11, 2688])),
    ("pnasnet_large", dict(Stem=[42, 540], **{"Cell_%d" % i: [42 if i < 4 else 21 if i < 8 else 11,
                                                               1080 if i < 4 else 2160 if i < 8 else 4320]
                                               for i in range(12)})),
])
def test_large_nasnet_endpoints(name, golden):
    B, nc = 1, 1000
    ep = {}
    nets_factory.build(name, nc)(torch.zeros(B, 331, 331, 3), training=True, end_points=ep)
    want = {k: [B, s, s, c] for k, (s, c) in golden.items()}
    want.update(global_pool=[B, 4032 if name == "nasnet_large" else 4320], AuxLogits=[B, nc], Logits=[B, nc],
                Predictions=[B, nc])
    _check_eps(ep, want)


def test_nasnet_reduction_layers():
    assert nasnet.calc_reduction_layers(18, 2) == [6, 12]
    assert nasnet.calc_reduction_layers(12, 2) == [4, 8]


# ---------------------------------------------------------------------------------------------
# classic nets: logits shapes
@pytest.mark.parametrize("name,size,nc", [("alexnet_v2", 224, 1000), ("overfeat", 231, 1000), ("vgg_a", 224, 1000),
                                          ("vgg_19", 224, 1000), ("resnet_v2_50", 224, 1000),
                                          ("mobilenet_v2", 224, 1001), ("inception_resnet_v2", 299, 1001)])
def test_logits_shape(name, size, nc):
    m = nets_factory.build(name, nc)
    with torch.no_grad():
        out = m(torch.zeros(1, size, size, 3), training=False)
    assert list(out.shape) == [1, nc]


# ---------------------------------------------------------------------------------------------
# GANs (dcgan_test.py, cyclegan_test.py, pix2pix_test.py)
def test_dcgan_generator_and_discriminator_graphs():
    for i, B in zip(range(3, 7), range(3, 8)):
        fs = 2 ** i
        (img, ep), _ = _run(gans.dcgan_generator, torch.randn(B, 64), depth=32, final_size=fs)
        assert list(img.shape) == [B, fs, fs, 3]
        assert set(ep) == {"deconv%d" % j for j in range(1, i)} | {"logits"}
        for j in range(1, i):
            assert ep["deconv%d" % j].shape[-1] == 32 * 2 ** (i - j - 1)
    for i, B in zip(range(1, 6), range(3, 8)):
        w = 2 ** i
        (out, ep), _ = _run(gans.dcgan_discriminator, torch.rand(B, w, w, 3) * 2 - 1, depth=32)
        assert list(out.shape) == [B, 1]
        assert set(ep) == {"conv%d" % j for j in range(1, i + 1)} | {"logits"}
        for j in range(1, i + 1):
            assert ep["conv%d" % j].shape[-1] == 32 * 2 ** (j - 1)
    with pytest.raises(ValueError):
        _run(gans.dcgan_generator, torch.randn(2, 64), final_size=4)
    with pytest.raises(ValueError):
        _run(gans.dcgan_discriminator, torch.randn(2, 28, 28, 3))


@pytest.mark.parametrize("shape,k", [((4, 32, 32, 3), 3), ((3, 128, 128, 3), 3), ((2, 80, 400, 3), 3),
                                     ((1, 32, 32, 3), 4), ((1, 32, 32, 3), 5), ((1, 32, 32, 3), 6)])
def test_cyclegan_generator_shapes(shape, k):
    (out, _), _ = _run(gans.cyclegan_generator_resnet, torch.ones(shape), kernel_size=k)
    assert tuple(out.shape) == shape


@pytest.mark.parametrize("h,w", [(29, 32), (30, 32), (31, 32), (32, 29), (32, 30), (32, 31)])
def test_cyclegan_requires_multiple_of_four(h, w):
    with pytest.raises(ValueError):
        _run(gans.cyclegan_generator_resnet, torch.ones(1, h, w, 3))


@pytest.mark.parametrize("method", ["nn_upsample_conv", "conv2d_transpose"])
def test_pix2pix_generator_output_size(method):
    blocks = [(64, 0.5), (128, 0)]  # reduced default blocks (pix2pix_test._reduced_default_blocks)

    def fn(x):
        with gans.pix2pix_arg_scope():
            return gans.pix2pix_generator(x, 4, blocks=blocks, upsample_method=method)
    (logits, ep), _ = _run(fn, torch.ones(2, 256, 256, 3))
    assert list(logits.shape) == [2, 256, 256, 4]
    assert len([k for k in ep if k.startswith("encoder")]) == 2
    assert len([k for k in ep if k.startswith("decoder")]) == 2


@pytest.mark.parametrize("pad", [2, 0])
def test_pix2pix_discriminator_four_layers(pad):
    def size(n, stride=2, k=4):
        return (n + 2 * pad - k) // stride + 1
    o = size(size(size(256)))
    o = size(size(o, 1), 1)

    def fn(x):
        with gans.pix2pix_arg_scope():
            return gans.pix2pix_discriminator(x, [64, 128, 256, 512], padding=pad)
    (logits, ep), _ = _run(fn, torch.ones(2, 256, 256, 3))
    assert list(logits.shape) == [2, o, o, 1] and list(ep["predictions"].shape) == [2, o, o, 1]


def test_mobilenet_v1_base_model_variable_count():
    # reference vgg/nets/mobilenet_v1_test.py:344-353 (testModelHasExpectedNumberOfParameters):
    # mobilenet_v1_base under arg_scope(conv2d / separable_conv2d, normalizer_fn=slim.batch_norm) -
    # weights + BN beta / moving_mean / moving_variance (slim BN default scale=False) = 3,217,920
    from distributed_tensorflow_models_amd.compat import slim as S

    def base(images, is_training=True, num_classes=None):
        ep = {}
        with S.arg_scope([S.conv2d, S.separable_conv2d], normalizer_fn=S.batch_norm):
            with S.variable_scope("MobilenetV1"):
                return slim_nets.mobilenet_v1_base(images, ep), ep

    m = SlimModel(base, 224)
    n = sum(p.numel() for p in m.parameters()) + sum(b.numel() for b in m.buffers())
    assert n == 3217920


def test_sibling_weight_groups_declared():
    """The merged-forward head groups the models declare (engine.prepare_compute_copies puts each group's bf16
    copies side by side): Inception-v3 - every mixed block except mixed_17x17x768a (one 1x1 head).  ResNet-50
    declares none (its merged projection forward measured slower and was removed)."""
    from distributed_tensorflow_models_amd.models import nets_factory
    inc = nets_factory.build("inception_v3_slim_old", num_classes=11)
    groups = inc.sibling_weight_groups()
    widths = [[w.shape[0] for w in g] for g in groups]
    assert len(groups) == 10
    assert widths[0] == [64, 48, 64, 32] and widths[3] == [192, 128, 128, 192] and widths[-1] == [320, 384, 448, 192]
    assert all(len({tuple(w.shape[1:]) for w in g}) == 1 for g in groups)
    rn = nets_factory.build("resnet_v1_50", num_classes=11)
    assert not hasattr(rn, "sibling_weight_groups")


def test_inception_v3_slim_old_endpoints():
    """End points of the old-slim Inception-v3 as /root/reference/inception/slim/inception_model.py:88-331 names
    them (shapes from its inception_test.py geometry at 299x299)."""
    B, nc = 2, 1001
    ep = {}
    m = nets_factory.build("inception_v3_slim_old", nc)
    logits, aux = m(torch.zeros(B, 299, 299, 3), training=True, end_points=ep)
    g = {'conv0': [B, 149, 149, 32], 'conv1': [B, 147, 147, 32], 'conv2': [B, 147, 147, 64],
         'pool1': [B, 73, 73, 64], 'conv3': [B, 73, 73, 80], 'conv4': [B, 71, 71, 192], 'pool2': [B, 35, 35, 192],
         'mixed_35x35x256a': [B, 35, 35, 256], 'mixed_35x35x288a': [B, 35, 35, 288],
         'mixed_35x35x288b': [B, 35, 35, 288], 'mixed_17x17x768a': [B, 17, 17, 768],
         'mixed_17x17x768b': [B, 17, 17, 768], 'mixed_17x17x768c': [B, 17, 17, 768],
         'mixed_17x17x768d': [B, 17, 17, 768], 'mixed_17x17x768e': [B, 17, 17, 768],
         'aux_logits': [B, nc], 'mixed_17x17x1280a': [B, 8, 8, 1280], 'mixed_8x8x2048a': [B, 8, 8, 2048],
         'mixed_8x8x2048b': [B, 8, 8, 2048], 'logits': [B, nc], 'predictions': [B, nc]}
    _check_eps(ep, g)
    assert list(aux.shape) == [B, nc] and list(logits.shape) == [B, nc]
