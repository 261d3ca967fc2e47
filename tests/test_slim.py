"""TF-Slim facade behaviour ported from the reference's old-slim unit tests (SURVEY.md C60:
inception/slim/{scopes,variables,losses,collections}_test.py) plus flags/train facades."""
import math

import pytest
import torch

from distributed_tensorflow_models_amd.compat import flags as tf_flags
from distributed_tensorflow_models_amd.compat import slim
from distributed_tensorflow_models_amd.compat import train as tf_train
from distributed_tensorflow_models_amd.models.inception_v3_slim import InceptionV3Slim
from distributed_tensorflow_models_amd.models.layers import tf_variables


@slim.add_arg_scope
def func1(*args, **kwargs):
    return args, kwargs


@slim.add_arg_scope
def func2(*args, **kwargs):
    return args, kwargs


@pytest.fixture(autouse=True)
def fresh_store():
    st = slim.VariableStore()
    with slim.use_store(st):
        yield st


# ---------------------------------------------------------------------------------------------
# scopes_test.py
def test_arg_scope_simple_overwrite_nested_shared():
    with slim.arg_scope([func1], a=1, b=None, c=[1]):
        assert func1(0) == ((0,), {"a": 1, "b": None, "c": [1]})
        assert func1(0, b=2) == ((0,), {"a": 1, "b": 2, "c": [1]})     # explicit kwargs win
        with slim.arg_scope([func1], b=2):                            # nested scope overrides
            assert func1(0) == ((0,), {"a": 1, "b": 2, "c": [1]})
        assert func1(0) == ((0,), {"a": 1, "b": None, "c": [1]})
    with slim.arg_scope((func1, func2), a=1, b=None, c=[1]):          # shared, tuple of ops
        assert func1(0) == func2(0) == ((0,), {"a": 1, "b": None, "c": [1]})
    with slim.arg_scope([func1, func2], a=1, b=None, c=[1]):          # partially shared
        with slim.arg_scope([func2], d=[2]):
            assert func1(0)[1] == {"a": 1, "b": None, "c": [1]}
            assert func2(0)[1] == {"a": 1, "b": None, "c": [1], "d": [2]}
    assert func1(0) == ((0,), {})


def test_arg_scope_reuse():
    with slim.arg_scope([func1], a=1, b=None, c=[1]) as scope1:
        with slim.arg_scope([func2], b=2, d=[2]) as scope2:
            pass
    with slim.arg_scope(scope1):
        assert func1(0)[1] == {"a": 1, "b": None, "c": [1]} and func2(0)[1] == {}
    with slim.arg_scope(scope2):
        assert func2(0)[1] == {"b": 2, "d": [2]} and func1(0)[1] == {"a": 1, "b": None, "c": [1]}


def test_arg_scope_rejects_undecorated():
    with pytest.raises(ValueError):
        with slim.arg_scope([math.sqrt], a=1):
            pass


# ---------------------------------------------------------------------------------------------
# variables_test.py
def test_create_get_reuse_variables():
    with slim.variable_scope("A"):
        a = slim.variable("a", [5])
        assert a.tf_name == "A/a" and tuple(a.shape) == (5,)
        assert slim.variable("a", [5]) is a                       # reuse by name
    with slim.variable_scope("B"):
        b = slim.variable("a", [5])
    assert slim.get_variables("A") == [a] and slim.get_variables("B") == [b]
    assert slim.get_variables(suffix="a") == [a, b]
    assert slim.get_variables_by_name("a") == [a, b]
    assert slim.get_variables_by_name("a", scope="B") == [b]


def test_variables_to_restore_and_collections():
    with slim.variable_scope("A"):
        a = slim.variable("a", [5])
    with slim.variable_scope("B"):
        b = slim.variable("a", [5], restore=False)
        c = slim.variable("c", [5], collections=["my_collection"])
    assert slim.get_variables_to_restore() == [a, c]
    assert slim.get_store().get_collection("my_collection") == [c]
    assert set(map(id, slim.get_variables())) == {id(a), id(b), id(c)}


def test_variable_initializers_and_regularizers():
    v = slim.variable("w", [4, 4], initializer=("constant", 0.5), regularizer=slim.l2_regularizer(0.1))
    assert torch.all(v == 0.5)
    assert v.weight_decay == pytest.approx(0.1)      # L2 becomes coupled decay in the optimizer
    reg = slim.losses.get_regularization_losses()
    assert len(reg) == 1 and reg[0].item() == pytest.approx(0.1 * 16 * 0.25 / 2)


def test_variable_device_chooser_round_robin():
    ch = slim.VariableDeviceChooser(num_parameter_servers=3)
    assert [ch() for _ in range(4)] == ["/job:ps/task:0/CPU:0", "/job:ps/task:1/CPU:0", "/job:ps/task:2/CPU:0",
                                        "/job:ps/task:0/CPU:0"]
    assert slim.VariableDeviceChooser()() == "CPU:0"
    setter = tf_train.replica_device_setter(ps_tasks=2)
    assert setter is not None


def test_default_scope_uniquification():
    x = torch.zeros(1, 8, 8, 8)
    slim.conv2d(x, 8, 3)
    slim.conv2d(x, 8, 3)
    names = sorted(v.tf_name for v in slim.get_variables())
    assert names == ["Conv/biases", "Conv/weights", "Conv_1/biases", "Conv_1/weights"]


# ---------------------------------------------------------------------------------------------
# losses_test.py
def test_l1_l2_losses_and_regularizers():
    t = torch.ones(5, 5, 5)
    n = 125
    assert slim.losses.l1_loss(t, 0.01).item() == pytest.approx(n * 0.01, abs=1e-5)
    assert slim.losses.l2_loss(t, 0.01).item() == pytest.approx(n * 0.01 / 2, abs=1e-5)
    assert slim.l1_regularizer()(t).item() == pytest.approx(n)
    assert slim.l1_regularizer(0.01)(t).item() == pytest.approx(n * 0.01)
    assert slim.l2_regularizer()(t).item() == pytest.approx(n / 2)
    assert slim.l2_regularizer(0.01)(t).item() == pytest.approx(n * 0.01 / 2)
    assert slim.l1_l2_regularizer()(t).item() == pytest.approx(n + n / 2)
    assert slim.l1_l2_regularizer(0.5, 0.1)(t).item() == pytest.approx(0.5 * n + 0.1 * n / 2)


def test_cross_entropy_loss():
    logits = torch.tensor([[10.0, 0.0, 0.0], [0.0, 10.0, 0.0], [0.0, 0.0, 10.0]])
    right = torch.eye(3)
    wrong = torch.tensor([[0, 0, 1], [1, 0, 0], [0, 1, 0]], dtype=torch.float32)
    assert slim.losses.cross_entropy_loss(logits, right).item() == pytest.approx(0.0, abs=1e-3)
    assert slim.losses.cross_entropy_loss(logits, wrong).item() == pytest.approx(10.0, abs=1e-3)
    assert slim.losses.cross_entropy_loss(logits, wrong, weight=0.5).item() == pytest.approx(5.0, abs=1e-3)
    # label smoothing: y*(1-e) + e/K
    e = 0.1
    ls = slim.losses.cross_entropy_loss(logits, right, label_smoothing=e).item()
    logp = torch.log_softmax(logits, -1)
    expect = -((right * (1 - e) + e / 3) * logp).sum(-1).mean().item()
    assert ls == pytest.approx(expect, rel=1e-4)
    assert len(slim.losses.get_losses()) == 4


# ---------------------------------------------------------------------------------------------
# collections_test.py (old-slim Inception-v3 variable layout)
def test_inception_v3_old_slim_collections():
    names = [n for n, *_ in tf_variables(InceptionV3Slim(1001))]
    assert len(names) == 388

    def by(name):
        return [n for n in names if n.split("/")[-1] == name]
    assert (len(by("weights")), len(by("biases")), len(by("beta")), len(by("gamma")), len(by("moving_mean")),
            len(by("moving_variance"))) == (98, 2, 96, 0, 96, 96)

    def scope(s):
        return [n for n in names if n.startswith(s + "/")]
    for s, k in (("conv0", 4), ("conv1", 4), ("conv2", 4), ("conv3", 4), ("conv4", 4), ("mixed_35x35x256a", 28),
                 ("mixed_35x35x288a", 28), ("mixed_35x35x288b", 28), ("mixed_17x17x768a", 16),
                 ("mixed_17x17x768b", 40), ("mixed_17x17x768c", 40), ("mixed_17x17x768d", 40),
                 ("mixed_17x17x768e", 40), ("mixed_8x8x2048a", 36), ("mixed_8x8x2048b", 36), ("logits", 2),
                 ("aux_logits", 10)):
        assert len(scope(s)) == k, s


# ---------------------------------------------------------------------------------------------
# tf.app.flags / tf.train facades
def test_flags_parse():
    F = tf_flags.FLAGS
    tf_flags.DEFINE_integer("t_int", 3, "")
    tf_flags.DEFINE_boolean("t_bool", False, "")
    tf_flags.DEFINE_string("t_str", "x", "")
    tf_flags.DEFINE_float("t_f", 1.5, "")
    rest = F.parse(["prog", "--t_int=5", "--t_bool", "--t_str", "y", "--t_f=2e-3", "--unknown=1"])
    assert (F.t_int, F.t_bool, F.t_str, F.t_f) == (5, True, "y", 0.002)
    assert rest == ["prog", "--unknown=1"]
    F.parse(["prog", "--not_bool"])          # "--no" + "t_bool"
    assert F.t_bool is False
    F.parse(["prog", "--t_int=1e7"])         # reference passes max_steps as 1e7
    assert F.t_int == 10000000
    with pytest.raises(AttributeError):
        F.t_missing


def test_exponential_decay_staircase_and_ema_decay():
    sched = tf_train.ExponentialDecay(0.1, 100, 0.5, staircase=True)
    assert sched(0) == pytest.approx(0.1) and sched(99) == pytest.approx(0.1) and sched(100) == pytest.approx(0.05)
    smooth = tf_train.ExponentialDecay(0.1, 100, 0.5, staircase=False)
    assert smooth(50) == pytest.approx(0.1 * 0.5 ** 0.5)
    ema = tf_train.ExponentialMovingAverage(0.9999)
    assert ema.effective_decay(0) == pytest.approx(0.1)       # min(decay, (1+n)/(10+n))
    assert ema.effective_decay(10 ** 7) == pytest.approx(0.9999)
