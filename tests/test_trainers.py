"""Entry scripts end-to-end on CPU: every trainer runs a few steps with the reference flags,
writes TF-layout checkpoints, resumes, and the evaluator restores EMA shadows (SURVEY.md §2.4,
C55-C59, §5.4)."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = "distributed_tensorflow_models_amd.trainers."


def _run(mod, *args, timeout=600):
    env = dict(os.environ, OMP_NUM_THREADS="4")
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, "-m", PKG + mod] + list(args), cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=timeout)
    assert p.returncode == 0, (p.stdout + p.stderr)[-4000:]
    return p.stdout + p.stderr


@pytest.mark.parametrize("mod,batch,style", [
    ("cifar10_cnn_bsp", 8, "cnn"), ("cifar10_alexnet_bsp", 4, "standard"), ("cifar10_vgg_bsp", 2, "standard"),
    ("cifar10_vgg_asp", 2, "standard"), ("cifar10_resnet_bsp", 4, "short"), ("cifar10_cifarnet_bsp", 8, "standard"),
    ("mnist_lenet_bsp", 8, "standard"), ("imagenet_inception_bsp", 1, "short"), ("imagenet_inception_ssp", 1, "short"),
    ("mobilenet_v1_train", 2, "short"),
])
def test_trainer_runs_and_checkpoints(tmp_path, mod, batch, style):
    d = str(tmp_path / "train")
    out = _run(mod, "--max_steps=2", "--batch_size=%d" % batch, "--train_dir=" + d, "--data_dir=/nonexistent",
               "--synthetic_data")
    line = [l for l in out.splitlines() if "step 1 " in l]
    assert line, out[-2000:]
    if style == "short":
        assert "(gs 2), loss= " in line[0] and "samples/s" in line[0]
    else:
        assert "(global_step 2), loss = " in line[0] and "examples/sec" in line[0]
        assert line[0].startswith("time: ") == (style == "standard")
    assert os.path.exists(os.path.join(d, "model.ckpt-2.index"))
    assert os.path.exists(os.path.join(d, "checkpoint"))


def test_resume_and_ema_eval(tmp_path):
    from distributed_tensorflow_models_amd.ckpt.bundle import BundleReader
    from distributed_tensorflow_models_amd import evaluator
    from distributed_tensorflow_models_amd.models import nets_factory
    d = str(tmp_path / "train")
    _run("cifar10_cnn_bsp", "--max_steps=2", "--batch_size=8", "--train_dir=" + d)
    out = _run("cifar10_cnn_bsp", "--max_steps=4", "--batch_size=8", "--train_dir=" + d)
    assert "restored" in out and "step 2 (global_step 3)" in out
    r = BundleReader(os.path.join(d, "model.ckpt-4"))
    names = set(r.names())
    # reference cnn layout: global step is the unnamed tf.Variable(0); EMA shadows for every weight
    assert "Variable" in names and int(r.get_tensor("Variable")) == 4
    assert "local3/weights/ExponentialMovingAverage" in names
    model = nets_factory.build("cifar10_cnn", 10)
    evaluator.restore_for_eval(model, os.path.join(d, "model.ckpt-4"), use_ema=True)
    ema = r.get_tensor("local3/weights/ExponentialMovingAverage")
    raw = r.get_tensor("local3/weights")
    assert not np.allclose(ema, raw)
    got = [p for p in model.parameters() if p.tf_name == "local3/weights"][0]
    np.testing.assert_allclose(got.detach().numpy().reshape(ema.shape), ema, rtol=0, atol=0)
    ev = _run("cifar10_cnn_eval", "--checkpoint_dir=" + d, "--eval_dir=" + str(tmp_path / "eval"), "--run_once",
              "--num_examples=16", "--batch_size=8")
    assert "precision @ 1 = " in ev and "global_step: 4" in ev
    assert any(f.startswith("events.out.tfevents") for f in os.listdir(tmp_path / "eval"))


def test_fresh_wipes_train_dir(tmp_path):
    d = str(tmp_path / "train")
    _run("cifar10_cifarnet_bsp", "--max_steps=2", "--batch_size=4", "--train_dir=" + d)
    out = _run("cifar10_cifarnet_bsp", "--max_steps=1", "--batch_size=4", "--train_dir=" + d, "--fresh")
    assert "restored" not in out
    assert not os.path.exists(os.path.join(d, "model.ckpt-2.index"))


def test_launcher_dry_run():
    from distributed_tensorflow_models_amd.parallel import launcher
    cmds, ev = launcher.build_commands("inception", "ssp", 8, ["--batch_size=32"], 29500, eval_=True)
    assert len(cmds) == 8 and cmds[7][2]["RANK"] == "7" and cmds[0][2]["MASTER_ADDR"] == "127.0.0.1"
    assert cmds[0][1][2].endswith("imagenet_inception_ssp")
    assert ev[1][2].endswith("imagenet_inception_eval")
    mod, extra = launcher.resolve("resnet", "asp")  # any model in any mode via --sync_mode
    assert mod == "cifar10_resnet_bsp" and extra == ["--sync_mode=asp"]


@pytest.mark.parametrize("mod,scope,gs,probe", [
    ("cifar10_alexnet_bsp", "partitioned_space/", "partitioned_space/Variable", "alexnet_v2/conv1/weights"),
    ("cifar10_cifarnet_bsp", "partitioned_space/", "partitioned_space/Variable", "CifarNet/conv1/weights"),
    ("cifar10_vgg_bsp", "root/", "root/Variable", "vgg_16/conv1/conv1_1/weights"),
    ("cifar10_resnet_bsp", "root/", "Variable", None),
])
def test_trainer_scopes_and_partitioned_layout(tmp_path, mod, scope, gs, probe):
    """SURVEY.md §5.4 name layout of the partitioned trainers: every variable under the trainer's
    variable_scope, saved as fixed_size_partitioner(len(ps_hosts)) slices; eval restores it."""
    from distributed_tensorflow_models_amd.ckpt.bundle import BundleReader
    d = str(tmp_path / "train")
    _run(mod, "--max_steps=1", "--batch_size=2", "--train_dir=" + d, "--data_dir=/nonexistent", "--synthetic_data",
         "--ps_hosts=127.0.0.1:1,127.0.0.1:2")
    r = BundleReader(os.path.join(d, "model.ckpt-1"))
    names = r.names()
    assert gs in names and int(r.get_tensor(gs)) == 1
    assert all(n.startswith(scope) or n == gs for n in names), names[:5]
    trainables = [n for n in names if n != gs and not n.endswith("ExponentialMovingAverage")]
    assert trainables and all(n in r.sliced for n in trainables if r.get_variable_to_shape_map()[n])
    if probe:
        assert scope + probe in names
        assert r.get_tensor(scope + probe).shape == tuple(r.get_variable_to_shape_map()[scope + probe])
    else:  # tf.layers auto-names under root/ (resnet/resnet_model.py)
        assert any(n.startswith("root/") and "batch_normalization" in n and "moving_mean" in n for n in names), names
    evm = mod.replace("_bsp", "_eval")
    ev = _run(evm, "--checkpoint_dir=" + d, "--eval_dir=" + str(tmp_path / "eval"), "--run_once",
              "--num_examples=4", "--batch_size=2", "--data_dir=/nonexistent", "--synthetic_data")
    assert "precision @ 1" in ev


def test_asp_checkpoint_keeps_optimizer_slots(tmp_path):
    """ASP: the momentum / RMSProp slots live in the owner shards and are checkpointed from there."""
    from distributed_tensorflow_models_amd.ckpt.bundle import BundleReader
    d = str(tmp_path / "train")
    _run("imagenet_inception_asp", "--max_steps=1", "--batch_size=1", "--train_dir=" + d, "--data_dir=/nonexistent",
         "--synthetic_data")
    r = BundleReader(os.path.join(d, "model.ckpt-1"))
    names = r.names()
    assert "conv0/weights/RMSProp" in names and "conv0/weights/RMSProp_1" in names
    ms = r.get_tensor("conv0/weights/RMSProp")
    assert not np.allclose(ms, 1.0)  # ms slot (init 1.0) was updated by the push, and saved from the shard


def test_training_tb_scalars(tmp_path):
    """The chief writes train-side TensorBoard scalars (learning_rate, total_loss (raw), its 0.9
    moving average total_loss) into train_dir (reference cnn/cifar10.py:309-335,361)."""
    d = str(tmp_path / "train")
    _run("cifar10_cnn_bsp", "--max_steps=3", "--batch_size=8", "--train_dir=" + d, "--data_dir=/nonexistent",
         "--synthetic_data")
    ev = [f for f in os.listdir(d) if f.startswith("events.out.tfevents")]
    assert ev
    blob = open(os.path.join(d, ev[0]), "rb").read()
    for tag in (b"learning_rate", b"total_loss (raw)", b"total_loss", b"images_per_sec"):
        assert tag in blob


def test_resnet_training_accuracy_probe(tmp_path):
    """ResNet-CIFAR: every --train_accuracy_every steps the chief logs the reference's line
    'evaluation: step - N; accuracy: X' for the training-mode network on a fed batch of distorted training
    images (resnet/cifar10_resnet_bsp.py:146-148; 10,000 images by default, 32 here)."""
    d = str(tmp_path / "train")
    out = _run("cifar10_resnet_bsp", "--max_steps=3", "--batch_size=4", "--train_dir=" + d, "--data_dir=/nonexistent",
               "--train_accuracy_every=2", "--train_accuracy_batch=32", "--resnet_size=8")
    lines = [l for l in out.splitlines() if "evaluation: step - " in l]
    assert len(lines) == 2 and "evaluation: step - 0; accuracy: " in lines[0] and "step - 2;" in lines[1], out[-2000:]
    acc = float(lines[0].rsplit("accuracy: ", 1)[1])
    assert 0.0 <= acc <= 1.0


def test_training_accuracy_probe_leaves_moving_statistics():
    from distributed_tensorflow_models_amd.data.synthetic import SyntheticImages
    from distributed_tensorflow_models_amd.engine import moving_average_buffers
    from distributed_tensorflow_models_amd.models import nets_factory
    from distributed_tensorflow_models_amd.trainer import train_accuracy_probe
    torch.manual_seed(0)
    model = nets_factory.build("cifar10_resnet_v2", num_classes=10, resnet_size=8)
    before = [b.clone() for b in moving_average_buffers(model)]
    acc = train_accuracy_probe(model, SyntheticImages(16, 32, 32, 3, 10, "cpu", dtype=torch.float32))
    assert 0.0 <= acc <= 1.0
    assert all(torch.equal(a, b) for a, b in zip(before, moving_average_buffers(model)))


def test_bsp_fine_tune_two_ranks_keeps_moving_statistics(tmp_path):
    """under BSP with 2 replicas, --fine_tune_checkpoint must be restored before the BN-statistics
    sync snapshot; restored after it, the first synced step folds the restore into the delta (init + W*(ckpt-init):
    moving_variance 1 + 2*(5-1) = 9 below).  The fine-tune checkpoint sets every moving mean to 3 and variance to 5;
    one BSP step at decay 0.997 must leave them near 3 / 5."""
    import socket
    from distributed_tensorflow_models_amd.ckpt.bundle import BundleReader, write_bundle
    base = str(tmp_path / "base")
    _run("cifar10_resnet_bsp", "--max_steps=1", "--batch_size=2", "--train_dir=" + base, "--data_dir=/nonexistent",
         "--synthetic_data", "--resnet_size=8")
    r = BundleReader(os.path.join(base, "model.ckpt-1"))
    tensors = {}
    for n in r.names():
        if n.endswith("ExponentialMovingAverage") or n == "Variable":
            continue
        t = np.asarray(r.get_tensor(n))
        if n.endswith("moving_mean"):
            t = np.full_like(t, 3.0)
        elif n.endswith("moving_variance"):
            t = np.full_like(t, 5.0)
        tensors[n] = t
    ft = str(tmp_path / "ft" / "model.ckpt-0")
    os.makedirs(os.path.dirname(ft))
    write_bundle(ft, tensors)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    d = str(tmp_path / "train")
    env = dict(os.environ, OMP_NUM_THREADS="2")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr=127.0.0.1", "--master-port=%d" % port, "-m", PKG + "cifar10_resnet_bsp",
                        "--max_steps=1", "--batch_size=2", "--train_dir=" + d, "--data_dir=/nonexistent",
                        "--synthetic_data", "--resnet_size=8", "--fine_tune_checkpoint=" + ft],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, (p.stdout + p.stderr)[-4000:]
    assert "fine-tuning from" in p.stdout + p.stderr
    out = BundleReader(os.path.join(d, "model.ckpt-1"))
    mm = [n for n in out.names() if n.endswith("moving_mean")]
    mv = [n for n in out.names() if n.endswith("moving_variance")]
    assert mm and mv
    for n in mm:
        v = np.asarray(out.get_tensor(n))
        assert np.all(np.abs(v - 3.0) < 0.5), (n, v[:4])
    for n in mv:
        v = np.asarray(out.get_tensor(n))
        assert np.all((v > 4.0) & (v < 6.0)), (n, v[:4])
