"""Old TF-Slim ``ops`` layer behaviour, ported as assertions from the reference's
inception/slim/ops_test.py (SURVEY.md §4.1 "layers", "BatchNorm numerics"; C42) and exercised
through ``compat.old_slim`` (CPU fp32 oracle path; the same calls run the HIP kernels on a GPU)."""
import numpy as np
import pytest
import torch

from distributed_tensorflow_models_amd.compat import old_slim as oslim
from distributed_tensorflow_models_amd.compat import slim

ops, variables, losses, scopes = oslim.ops, oslim.variables, oslim.losses, oslim.scopes


@pytest.fixture(autouse=True)
def fresh_store():
    st = slim.VariableStore()
    with slim.use_store(st):
        yield st


def _names(scope=None):
    return sorted(v.tf_name for v in variables.get_variables(scope))


def _images(h=3, w=3, c=3, n=5, seed=0):
    return torch.rand(n, h, w, c, generator=torch.Generator().manual_seed(seed))


# ---------------------------------------------------------------------------------------------
# ConvTest
@pytest.mark.parametrize("kernel,stride,padding,out_hw", [
    ([3, 3], 1, "SAME", (3, 3)), (3, 1, "SAME", (3, 3)), ([3, 1], 1, "SAME", (3, 3)), ([1, 3], 1, "SAME", (3, 3)),
    ([3, 3], 2, "SAME", (2, 2)), ([3, 3], 1, "VALID", (1, 1)),
])
def test_conv_shapes(kernel, stride, padding, out_hw):
    y = ops.conv2d(_images(), 32, kernel, stride=stride, padding=padding)
    assert list(y.shape) == [5, out_hw[0], out_hw[1], 32]
    assert (y >= 0).all()  # default activation is ReLU


def test_conv_creates_weights_and_biases_vars_and_scope():
    assert _names() == []
    ops.conv2d(_images(), 32, [3, 3], scope="conv")
    assert _names() == ["conv/biases", "conv/weights"]
    assert list(variables.get_unique_variable("conv/weights").shape) == [32, 3, 3, 3]  # HWIO [3,3,3,32] exported


def test_conv_without_activation_and_stddev():
    y = ops.conv2d(_images(), 32, [3, 3], activation=None, stddev=1.0)
    assert (y < 0).any()


@pytest.mark.parametrize("wd,nreg", [(0.01, 1), (0, 0)])
def test_conv_weight_decay(wd, nreg):
    ops.conv2d(_images(), 32, [3, 3], weight_decay=wd)
    assert len(losses.get_regularization_losses()) == nreg


def test_conv_reuse_and_nonreuse_vars():
    x = _images()
    ops.conv2d(x, 32, [3, 3], scope="conv1", weight_decay=0.01)
    ops.conv2d(x, 32, [3, 3], scope="conv1", reuse=True, weight_decay=0.01)
    assert len(variables.get_variables()) == 2
    assert len(losses.get_regularization_losses()) == 1
    ops.conv2d(x, 32, [3, 3])
    ops.conv2d(x, 32, [3, 3])
    assert _names() == ["Conv/biases", "Conv/weights", "Conv_1/biases", "Conv_1/weights", "conv1/biases",
                        "conv1/weights"]


def test_conv_with_batch_norm():
    x = _images()
    y = ops.conv2d(x, 32, [3, 3], batch_norm_params={"decay": 0.9})
    assert list(y.shape) == [5, 3, 3, 32]
    assert len(slim.get_store().get_collection("moving_vars")) == 2
    assert len(variables.get_variables("Conv/BatchNorm")) == 3
    assert "Conv/biases" not in _names()
    ops.conv2d(x, 32, [3, 3], batch_norm_params={"decay": 0.9}, scope="conv", )
    ops.conv2d(x, 32, [3, 3], batch_norm_params={"decay": 0.9}, scope="conv", reuse=True)
    assert len(variables.get_variables("conv/BatchNorm")) == 3


# ---------------------------------------------------------------------------------------------
# FCTest
def test_fc_create_vars_activation_wd_and_bn():
    x = torch.rand(5, 30)
    y = ops.fc(x, 32, scope="fc")
    assert list(y.shape) == [5, 32] and (y >= 0).all()
    assert _names() == ["fc/biases", "fc/weights"]
    assert list(variables.get_unique_variable("fc/weights").shape) == [30, 32]
    ops.fc(x, 32, weight_decay=0.01, scope="fc_wd")
    ops.fc(x, 32, weight_decay=0.01, scope="fc_wd", reuse=True)
    assert len(losses.get_regularization_losses()) == 1
    z = ops.fc(x, 32, activation=None, stddev=1.0)
    assert (z < 0).any()
    ops.fc(x, 32, batch_norm_params={"decay": 0.9}, scope="fc_bn")
    assert len(variables.get_variables("fc_bn/BatchNorm")) == 3
    assert ops.fc(torch.rand(5, 3, 3, 3), 7).shape == (5, 7)  # inputs are flattened


# ---------------------------------------------------------------------------------------------
# MaxPoolTest / AvgPoolTest
@pytest.mark.parametrize("pool", [ops.max_pool, ops.avg_pool])
@pytest.mark.parametrize("kernel,kw,out_hw", [
    ([3, 3], {}, 1), (3, {}, 1), ([3, 3], {"padding": "SAME"}, 2), ([3, 3], {"padding": "SAME", "stride": 1}, 3),
])
def test_pool_shapes(pool, kernel, kw, out_hw):
    y = pool(_images(), kernel, **kw)
    assert list(y.shape) == [5, out_hw, out_hw, 3]


@pytest.mark.parametrize("pool,red", [(ops.max_pool, torch.amax), (ops.avg_pool, torch.mean)])
def test_global_pool(pool, red):
    x = _images()
    y = pool(x, x.shape[1:3], stride=1)
    assert list(y.shape) == [5, 1, 1, 3]
    torch.testing.assert_close(y[:, 0, 0], red(x, dim=(1, 2)))


# ---------------------------------------------------------------------------------------------
# OneHotEncodingTest / DropoutTest / FlattenTest / repeat_op
def test_one_hot_encoding():
    y = ops.one_hot_encoding(torch.tensor([0, 1, 2]), 3)
    assert y.dtype == torch.float32 and torch.equal(y, torch.eye(3))
    assert list(ops.one_hot_encoding(torch.tensor([1, 0]), 5).shape) == [2, 5]


def test_dropout_training_and_inference():
    x = torch.ones(5, 3, 3, 3)
    y = ops.dropout(x, keep_prob=0.5)
    assert y.shape == x.shape and not torch.equal(y, x)
    assert set(torch.unique(y).tolist()) <= {0.0, 2.0}
    assert ops.dropout(x, is_training=False) is x


@pytest.mark.parametrize("shape,out", [((5, 3, 3, 3), (5, 27)), ((5, 3, 3), (5, 9)), ((7, 2), (7, 2))])
def test_flatten(shape, out):
    assert tuple(ops.flatten(torch.zeros(shape)).shape) == out
    with pytest.raises(ValueError):
        ops.flatten(torch.zeros(3))


def test_repeat_op_scopes():
    y = ops.repeat_op(3, _images(), ops.conv2d, 8, [3, 3], scope="conv1")
    assert list(y.shape) == [5, 3, 3, 8]
    assert _names() == ["conv1/Conv/biases", "conv1/Conv/weights", "conv1/Conv_1/biases", "conv1/Conv_1/weights",
                        "conv1/Conv_2/biases", "conv1/Conv_2/weights"]


def test_arg_scope_applies_to_old_ops():
    with scopes.arg_scope([ops.conv2d], stddev=0.1, weight_decay=0.004, padding="VALID"):
        y = ops.conv2d(_images(), 4, [3, 3])
    assert list(y.shape) == [5, 1, 1, 4]
    assert len(losses.get_regularization_losses()) == 1


# ---------------------------------------------------------------------------------------------
# BatchNormTest
@pytest.mark.parametrize("kw,expect", [
    ({}, ["BatchNorm/beta", "BatchNorm/moving_mean", "BatchNorm/moving_variance"]),
    ({"scale": True}, ["BatchNorm/beta", "BatchNorm/gamma", "BatchNorm/moving_mean", "BatchNorm/moving_variance"]),
    ({"center": False, "scale": True}, ["BatchNorm/gamma", "BatchNorm/moving_mean", "BatchNorm/moving_variance"]),
    ({"center": False, "scale": False}, ["BatchNorm/moving_mean", "BatchNorm/moving_variance"]),
])
def test_batch_norm_variables(kw, expect):
    y = ops.batch_norm(_images(), **kw)
    assert y.shape == (5, 3, 3, 3)
    assert _names() == expect
    trainable = sorted(v.tf_name for v in slim.trainable_variables())
    assert trainable == [n for n in expect if "moving" not in n]
    mv = slim.get_store().get_collection("moving_vars")
    assert sorted(v.tf_name for v in mv) == ["BatchNorm/moving_mean", "BatchNorm/moving_variance"]


def test_batch_norm_update_ops_and_reuse():
    x = _images()
    ops.batch_norm(x, scope="bn")
    assert slim.get_store().get_collection(oslim.UPDATE_OPS_COLLECTION) == ["bn/AssignMovingAvg",
                                                                           "bn/AssignMovingAvg_1"]
    ops.batch_norm(x, scale=True, scope="bn2")
    ops.batch_norm(x, scale=True, scope="bn2", reuse=True)
    assert len(variables.get_variables("bn2")) == 4
    ops.batch_norm(x, is_training=False, scope="bn3")
    assert "bn3/AssignMovingAvg" not in slim.get_store().get_collection(oslim.UPDATE_OPS_COLLECTION)


def test_batch_norm_compute_moving_vars():
    """10 training updates with decay 0.1 converge to the (biased) batch moments (ops_test.py:591-618)."""
    x = (torch.rand(10, 3, 3, 3, generator=torch.Generator().manual_seed(3)) * 4 + 2)
    for _ in range(10):
        ops.batch_norm(x, decay=0.1, scope="bn")
    mean = x.double().mean(dim=(0, 1, 2))
    var = x.double().var(dim=(0, 1, 2), unbiased=False)
    mm = variables.get_unique_variable("bn/moving_mean")
    mv = variables.get_unique_variable("bn/moving_variance")
    np.testing.assert_allclose(mm.detach().double().numpy(), mean.numpy(), rtol=1e-5)
    np.testing.assert_allclose(mv.detach().double().numpy(), var.numpy(), rtol=1e-5)


def test_batch_norm_eval_uses_and_keeps_moving_vars():
    """is_training=False normalises with the moving statistics and leaves them unchanged
    (ops_test.py:620-651)."""
    x = torch.rand(10, 3, 3, 3, generator=torch.Generator().manual_seed(4))
    ops.batch_norm(x, decay=0.1, is_training=False, scope="bn")
    mm = variables.get_unique_variable("bn/moving_mean")
    mv = variables.get_unique_variable("bn/moving_variance")
    with torch.no_grad():
        mm.copy_(torch.tensor([0.5, 0.25, 0.1]))
        mv.copy_(torch.tensor([2.0, 1.0, 0.5]))
    y = ops.batch_norm(x, decay=0.1, is_training=False, scope="bn")
    want = (x - mm.detach()) / torch.sqrt(mv.detach() + 0.001)
    torch.testing.assert_close(y, want)
    assert mm.tolist() == pytest.approx([0.5, 0.25, 0.1]) and mv.tolist() == pytest.approx([2.0, 1.0, 0.5])


# ---------------------------------------------------------------------------------------------
# old-slim losses keyword names (losses_test.py)
def test_old_losses_api():
    t = torch.ones(4, 4)
    assert losses.l2_regularizer(weight=0.1)(t).item() == pytest.approx(0.1 * 16 / 2)
    assert losses.l1_regularizer(weight=0.5)(t).item() == pytest.approx(8.0)
    assert losses.l1_l2_regularizer(weight_l1=1.0, weight_l2=2.0)(t).item() == pytest.approx(16 + 16)
    assert losses.l2_loss(t, weight=2.0).item() == pytest.approx(16.0)
    assert oslim.LOSSES_COLLECTION == "_losses" and oslim.UPDATE_OPS_COLLECTION == "_update_ops_"
