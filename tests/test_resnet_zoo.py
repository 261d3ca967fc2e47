"""ResNet v1 / v2 structure and atrous (output_stride) goldens, ported as assertions from the
reference's zoo tests (vgg/nets/resnet_v1_test.py:29-560, vgg/nets/resnet_v2_test.py) -- SURVEY.md
§4.4 "ResNet v1/v2 block shapes" and "conv2d_same even/odd equivalence".  CPU, fp32 oracle path
(the same model code runs the HIP kernels on the GPU); the dilated-conv decomposition itself is
checked against a direct dilated conv here and on the HIP kernels in tests/test_kernels_gpu.py.
"""
import numpy as np
import pytest
import torch

from distributed_tensorflow_models_amd.compat import slim
from distributed_tensorflow_models_amd.models import resnet_v1, slim_nets
from distributed_tensorflow_models_amd.ops import nn as F
from distributed_tensorflow_models_amd.ops import reference as ref


def create_test_input(batch, height, width, channels):
    """Mesh-grid fixture of resnet_v1_test.create_test_input: x[n, h, w, c] = h + w."""
    g = np.arange(height).reshape(height, 1) + np.arange(width).reshape(1, width)
    return torch.tensor(np.tile(g.reshape(1, height, width, 1), (batch, 1, 1, channels)), dtype=torch.float32)


# ---------------------------------------------------------------------------------------------
# resnet_utils
def test_subsample_three_by_three_and_four_by_four():
    x = torch.arange(9, dtype=torch.float32).reshape(1, 3, 3, 1)
    assert resnet_v1.subsample(x, 2).flatten().tolist() == [0, 2, 6, 8]
    x = torch.arange(16, dtype=torch.float32).reshape(1, 4, 4, 1)
    assert resnet_v1.subsample(x, 2).flatten().tolist() == [0, 2, 8, 10]


@pytest.mark.parametrize("n,y1,y4", [
    (4, [[14, 28, 43, 26], [28, 48, 66, 37], [43, 66, 84, 46], [26, 37, 46, 22]], [[48, 37], [37, 22]]),
    (5, [[14, 28, 43, 58, 34], [28, 48, 66, 84, 46], [43, 66, 84, 102, 55], [58, 84, 102, 120, 64],
         [34, 46, 55, 64, 30]], None),
])
def test_conv2d_same_even_odd(n, y1, y4):
    """conv2d_same(stride 2) == SAME conv subsampled; plain SAME stride-2 conv differs for even n
    (resnet_v1_test.py:72-160 goldens)."""
    x = create_test_input(1, n, n, 1)
    w = create_test_input(1, 3, 3, 1).reshape(3, 3, 1, 1).permute(3, 0, 1, 2).contiguous()  # HWIO -> KRSC
    r1 = F.conv2d(x, w, torch.zeros(1), 1, "SAME", relu=True)
    assert r1[0, :, :, 0].tolist() == y1
    r2 = resnet_v1.subsample(r1, 2)
    r3 = F.conv2d(x, w, torch.zeros(1), 2, resnet_v1.conv2d_same_padding(3, 2), relu=True)
    assert torch.equal(r3, r2)
    r4 = F.conv2d(x, w, torch.zeros(1), 2, "SAME", relu=True)
    assert r4[0, :, :, 0].tolist() == (y4 if y4 is not None else r2[0, :, :, 0].tolist())


@pytest.mark.parametrize("H,W,C,K,R,rate,padding", [
    (9, 9, 3, 4, 3, 2, "SAME"), (10, 7, 5, 3, 3, 2, "SAME"), (11, 11, 2, 2, 3, 4, "SAME"),
    (12, 12, 4, 6, 3, 3, "VALID"), (8, 13, 3, 2, 5, 2, "SAME"), (9, 9, 2, 3, 1, 2, "SAME"),
    (17, 17, 3, 5, 3, 2, (2, 2)),
])
def test_atrous_conv_space_to_batch_matches_dilated_conv(H, W, C, K, R, rate, padding):
    torch.manual_seed(0)
    x = torch.randn(2, H, W, C)
    w = torch.randn(K, R, R, C)
    b = torch.randn(K)
    want = ref.conv2d(x, w, b, 1, padding, True, rate)
    got = F._atrous_conv2d(x, w, b, 1, padding, True, rate)
    assert got.shape == want.shape
    torch.testing.assert_close(got, want, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("output_stride,ok", [(1, True), (2, True), (4, True), (8, True), (16, False), (3, False)])
def test_stack_blocks_plan_rates_and_errors(output_stride, ok):
    """Units past the target stride run stride 1 with the skipped strides folded into the rate."""
    blocks = [(1, 2, 2), (2, 2, 2), (4, 2, 2), (8, 2, 1)]
    if not ok:
        with pytest.raises(ValueError):
            resnet_v1.stack_blocks_plan(blocks, output_stride)
        return
    plan = resnet_v1.stack_blocks_plan(blocks, output_stride)
    stride = 1
    for units, sub in plan:
        for s, rate in units:
            assert s == 1 or rate == 1
            stride *= s
        assert sub == 1
    assert stride == output_stride
    dense = resnet_v1.stack_blocks_plan(blocks, None)
    assert [u for u, _ in dense] == [[(1, 1), (2, 1)]] * 3 + [[(1, 1), (1, 1)]]
    if output_stride == 2:
        assert plan[1][0] == [(1, 1), (1, 1)] and plan[2][0] == [(1, 2), (1, 2)] and plan[3][0] == [(1, 4), (1, 4)]


def test_store_non_strided_activations_moves_stride_to_block_end():
    plan = resnet_v1.stack_blocks_plan([(1, 2, 2), (2, 2, 1)], None, store_non_strided_activations=True)
    assert plan == [([(1, 1), (1, 1)], 2), ([(1, 1), (1, 1)], 1)]


# ---------------------------------------------------------------------------------------------
# complete small networks (resnet_v1_test.ResnetCompleteNetworkTest._resnet_small)
SMALL = [(1, 3, 2), (2, 3, 2), (4, 3, 2), (8, 2, 1)]


def _small_v1(num_classes=None, global_pool=True, output_stride=None, include_root_block=True,
              spatial_squeeze=True, scope="resnet"):
    torch.manual_seed(0)
    return resnet_v1.ResNetV1(num_classes=num_classes, global_pool=global_pool, spatial_squeeze=spatial_squeeze,
                              scope=scope, blocks=SMALL, include_root_block=include_root_block,
                              output_stride=output_stride)


def _run_v1(net, x, training=True):
    ep = {}
    with torch.no_grad():
        out = net(x, training=training, end_points=ep)
    return out, ep


def _run_v2(x, store=None, training=True, **kw):
    st = store or slim.VariableStore()
    st.training = training
    with slim.use_store(st), torch.no_grad():
        slim.begin_pass()
        out, ep = slim_nets.resnet_v2(x, blocks=SMALL, scope=kw.pop("scope", "resnet"), **kw)
    return out, ep, st


def _expected_names(version):
    exp = ["resnet/conv1"]
    for block in range(1, 5):
        for unit in range(1, 4 if block < 4 else 3):
            for conv in range(1, 4):
                exp.append("resnet/block%d/unit_%d/bottleneck_v%d/conv%d" % (block, unit, version, conv))
            exp.append("resnet/block%d/unit_%d/bottleneck_v%d" % (block, unit, version))
        exp.append("resnet/block%d/unit_1/bottleneck_v%d/shortcut" % (block, version))
        exp.append("resnet/block%d" % block)
    return sorted(exp + ["global_pool", "resnet/logits", "resnet/spatial_squeeze", "predictions"])


@pytest.mark.parametrize("version", [1, 2])
def test_endpoint_names(version):
    x = create_test_input(2, 224, 224, 3)
    if version == 1:
        _, ep = _run_v1(_small_v1(10), x)
    else:
        _, ep, _ = _run_v2(x, num_classes=10)
    assert sorted(ep) == _expected_names(version)


@pytest.mark.parametrize("version", [1, 2])
def test_classification_endpoints(version):
    x = create_test_input(2, 224, 224, 3)
    if version == 1:
        logits, ep = _run_v1(_small_v1(10, spatial_squeeze=False), x)
    else:
        logits, ep, _ = _run_v2(x, num_classes=10, spatial_squeeze=False)
    assert list(logits.shape) == [2, 1, 1, 10]
    assert list(ep["predictions"].shape) == [2, 1, 1, 10]
    assert list(ep["global_pool"].shape) == [2, 1, 1, 32]


@pytest.mark.parametrize("version", [1, 2])
@pytest.mark.parametrize("size,kw,shapes", [
    (224, dict(num_classes=10), [28, 14, 7, 7]),
    (321, dict(num_classes=10, global_pool=False, spatial_squeeze=False), [41, 21, 11, 11]),
    (128, dict(num_classes=10, global_pool=False, spatial_squeeze=False, include_root_block=False), [64, 32, 16, 16]),
    (321, dict(num_classes=10, global_pool=False, spatial_squeeze=False, output_stride=8), [41, 41, 41, 41]),
])
def test_block_endpoint_shapes(version, size, kw, shapes):
    x = create_test_input(2, size, size, 3)
    if version == 1:
        _, ep = _run_v1(_small_v1(**kw), x)
    else:
        _, ep, _ = _run_v2(x, **kw)
    for i, (hw, d) in enumerate(zip(shapes, [4, 8, 16, 32])):
        assert list(ep["resnet/block%d" % (i + 1)].shape) == [2, hw, hw, d]


@pytest.mark.parametrize("version", [1, 2])
@pytest.mark.parametrize("output_stride,hw", [(None, 3), (8, 9)])
def test_fully_convolutional_output_size(version, output_stride, hw):
    x = create_test_input(2, 65, 65, 3)
    if version == 1:
        out, _ = _run_v1(_small_v1(None, global_pool=False, output_stride=output_stride), x)
    else:
        out, _, _ = _run_v2(x, num_classes=None, global_pool=False, output_stride=output_stride)
    assert list(out.shape) == [2, hw, hw, 32]


@pytest.mark.parametrize("version", [1, 2])
def test_unknown_batch_size_logits(version):
    for batch in (1, 3):
        x = create_test_input(batch, 65, 65, 3)
        if version == 1:
            logits, _ = _run_v1(_small_v1(10, spatial_squeeze=False), x)
        else:
            logits, _, _ = _run_v2(x, num_classes=10, spatial_squeeze=False)
        assert list(logits.shape) == [batch, 1, 1, 10]


@pytest.mark.parametrize("version", [1, 2])
@pytest.mark.parametrize("output_stride", [4, 8, 16, 32, None])
def test_atrous_fully_convolutional_values(version, output_stride):
    """Dense (atrous) feature extraction subsampled == extraction at the nominal stride, same
    weights, inference-mode BN (resnet_v1_test.testAtrousFullyConvolutionalValues)."""
    x = create_test_input(2, 81, 81, 3)
    factor = 1 if output_stride is None else 32 // output_stride
    if version == 1:
        dense = _small_v1(None, global_pool=False, output_stride=output_stride, scope="resnet_v1_small")
        nominal = _small_v1(None, global_pool=False, scope="resnet_v1_small")
        nominal.load_state_dict(dense.state_dict())
        with torch.no_grad():
            for m in (dense, nominal):  # non-trivial inference BN statistics
                for name, b in m.named_buffers():
                    g = torch.Generator().manual_seed(len(name))
                    b.copy_(torch.rand(b.shape, generator=g) + (0.5 if "variance" in name else -0.5))
        out, _ = _run_v1(dense, x, training=False)
        want, _ = _run_v1(nominal, x, training=False)
    else:
        out, _, st = _run_v2(x, training=False, num_classes=None, global_pool=False, output_stride=output_stride)
        want, _, _ = _run_v2(x, store=st, training=False, num_classes=None, global_pool=False)
    out = resnet_v1.subsample(out, factor)
    assert out.shape == want.shape
    torch.testing.assert_close(out, want, rtol=1e-4, atol=1e-4 * float(want.abs().max()))


def test_resnet_v1_50_output_stride_16_shapes():
    """Full-size slim geometry in dense mode (FCN, output_stride 16 -> 321x321 input gives 21x21)."""
    net = resnet_v1.ResNetV1(50, num_classes=None, global_pool=False, output_stride=16)
    ep = {}
    with torch.no_grad():
        out = net(create_test_input(1, 321, 321, 3) / 100.0, training=False, end_points=ep)
    assert list(out.shape) == [1, 21, 21, 2048]
    assert [list(ep["resnet_v1_50/block%d" % i].shape)[1:3] for i in range(1, 5)] == [[41, 41], [21, 21],
                                                                                     [21, 21], [21, 21]]


@pytest.mark.parametrize("kernel,stride,rate,H", [(4, 2, 1, 9), (2, 2, 1, 8), (4, 2, 2, 11), (3, 2, 1, 10)])
def test_conv2d_same_even_kernel(kernel, stride, rate, H):
    """resnet_utils.conv2d_same for an even effective kernel: tf.pad [beg, end] (end = beg + 1) then
    VALID (reference vgg/nets/resnet_utils.py:77-122, ResnetUtilsTest.testConv2DSameEven's point)."""
    import torch.nn.functional as tF
    from distributed_tensorflow_models_amd.models.resnet_v1 import conv2d_same_padding
    from distributed_tensorflow_models_amd.ops import reference as ref
    torch.manual_seed(0)
    x = torch.randn(2, H, H, 8)
    w = torch.randn(16, kernel, kernel, 8)
    pad = conv2d_same_padding(kernel, stride, rate)
    keff = kernel + (kernel - 1) * (rate - 1)
    beg = (keff - 1) // 2
    end = keff - 1 - beg
    got = ref.conv2d(x, w, None, stride, pad, False, rate)
    xp = tF.pad(x, (0, 0, beg, end, beg, end))
    want = ref.conv2d(xp, w, None, stride, "VALID", False, rate)
    assert got.shape == want.shape
    torch.testing.assert_close(got, want)
