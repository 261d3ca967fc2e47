"""Checkpoint-polling evaluator behind every reference eval script.

Reference behaviour kept: poll ``checkpoint_dir`` every ``eval_interval_secs``, restore the newest
checkpoint (EMA shadows for trainable variables when the trainer keeps them - cnn/cifar10_eval.py:
128-135, inception/inception_eval.py:157-160), run ``ceil(num_examples / batch_size)`` batches,
print ``precision @ 1`` (+ ``recall @ 5`` for ImageNet, inception_eval.py:105-127) and write a TF
event summary to ``eval_dir``.  Reference defects fixed: the checkpoint state is re-read on every
poll (C56/C57 read it once), ResNet eval runs in inference mode (C58 used is_training=True), a
checkpoint already evaluated is not re-evaluated.
"""
import math
import os
import shutil
import time
from datetime import datetime

import torch

from . import trainer
from .ckpt.saver import Saver, TFVar, get_checkpoint_state, step_from_path
from .models.layers import tf_variables
from .ops import elementwise as E
from .utils.tb import SummaryWriter

EVAL_DEFAULTS = {
    # preset: (eval_dir, checkpoint_dir, interval, num_examples, use_ema, top5)
    "cnn": ("/home/ubuntu/cifar10/eval", "/home/ubuntu/cifar10/train", 60, 10000, True, False),
    "alexnet": ("/home/ubuntu/cifar10/eval", "/home/ubuntu/cifar10/train", 60, 1000, False, False),
    "vgg": ("/home/ubuntu/cifar10/eval", "/home/ubuntu/cifar10_train", 60, 1000, False, False),
    "vgg_asp": ("/home/ubuntu/cifar10/eval", "/home/ubuntu/cifar10_train", 60, 1000, False, False),
    "resnet": ("/home/ubuntu/cifar10/eval", "/home/ubuntu/cifar10/train", 60, 1000, False, False),
    "cifarnet": ("/home/ubuntu/cifar10/eval", "/home/ubuntu/cifar10/train", 60, 1000, False, False),
    "inception": ("/home/ubuntu/imagenet/eval", "/home/ubuntu/imagenet/train/", 300, 200, True, True),
    "resnet50": ("/tmp/resnet50_eval", "/tmp/resnet50_train", 300, 1000, False, True),
    "mobilenet_v1": ("/tmp/mobilenet_v1_eval", "/tmp/mobilenet_v1_train", 300, 50000, False, True),
    "lenet": ("/tmp/lenet_eval", "/tmp/lenet_train", 60, 1000, False, False),
}


def define_eval_flags(flags, preset):
    d = EVAL_DEFAULTS[preset]
    p = trainer.PRESETS[preset]
    F = flags.FLAGS
    for name, fn, default, h in (
            ("eval_dir", flags.DEFINE_string, d[0], "Directory where to write event logs."),
            ("eval_data", flags.DEFINE_string, "test", "Either 'test' or 'train_eval'."),
            ("subset", flags.DEFINE_string, "validation", "Either 'validation' or 'train' (ImageNet)."),
            ("checkpoint_dir", flags.DEFINE_string, d[1], "Directory where to read model checkpoints."),
            ("eval_interval_secs", flags.DEFINE_integer, d[2], "How often to run the eval."),
            ("num_examples", flags.DEFINE_integer, d[3], "Number of examples to run."),
            ("run_once", flags.DEFINE_boolean, False, "Whether to run eval only once."),
            ("batch_size", flags.DEFINE_integer, p["batch_size"], "Number of images to process in a batch."),
            ("data_dir", flags.DEFINE_string, p["data_dir"], "Path to the data directory."),
            ("resnet_size", flags.DEFINE_integer, 32, "The size of the ResNet model to use."),
            ("use_ema", flags.DEFINE_boolean, d[4], "restore ExponentialMovingAverage shadows"),
            ("synthetic_data", flags.DEFINE_boolean, False, "evaluate on synthetic batches"),
            ("max_evals", flags.DEFINE_integer, 0, "stop after N evaluations (0 = forever)"),
    ):
        fn(name, default, h)
        F.reset(name)


def restore_for_eval(model, path, use_ema, prefix=""):
    """With ``use_ema`` every variable that has a shadow (trainables and BN moving statistics, as
    tf.train.ExponentialMovingAverage.variables_to_restore maps them; reference
    cnn/cifar10_eval.py:132-135, inception/inception_eval.py:157-160) is restored from
    ``<v>/ExponentialMovingAverage``; everything else by name.  ``prefix``: the trainer's variable
    scope (the reference evals rebuild the net under it: alexnet/cifar10_alexnet_eval.py:125,
    resnet/cifar10_resnet_eval.py:107); partitioned (sliced) checkpoint entries are reassembled."""
    from .ckpt.bundle import BundleReader
    names = set(BundleReader(path).names()) if use_ema else set()
    vs = []
    for name, t, layout, trainable in tf_variables(model):
        name = prefix + name
        shadow = name + "/ExponentialMovingAverage"
        vs.append(TFVar(shadow if (use_ema and shadow in names) else name, t, layout))
    Saver(vs).restore(path)
    from .ops.nn import invalidate_weight_copies
    invalidate_weight_copies(model.parameters())


def _inputs(preset, flags, device):
    F = flags.FLAGS
    cfg = trainer.PRESETS[preset]
    S = cfg["image_size"]
    if cfg["dataset"] == "cifar10" and not F.synthetic_data:
        from .data import cifar10
        return cifar10.inputs(F.eval_data == "test", F.data_dir, F.batch_size, S, device=device)
    if cfg["dataset"] == "imagenet" and not F.synthetic_data:
        from .data import imagenet
        if torch.device(device).type == "cuda":
            from .data import imagenet_gpu
            return imagenet_gpu.inputs(imagenet.ImagenetData(F.subset, F.data_dir), F.batch_size, image_size=S,
                                       device=device)
        return imagenet.inputs(imagenet.ImagenetData(F.subset, F.data_dir), F.batch_size, image_size=S,
                               device=device)
    from .data.synthetic import SyntheticImages
    return SyntheticImages(F.batch_size, S, S, 1 if cfg["dataset"] == "synthetic_mnist" else 3,
                           cfg["num_classes"], device, seed=1234)


@torch.no_grad()
def eval_once(model, data, num_examples, batch_size, top5=False):
    num_iter = int(math.ceil(num_examples / float(batch_size)))
    c1 = c5 = 0
    for _ in range(num_iter):
        x, y = data.next_batch()
        out = model(x, training=False)
        if isinstance(out, tuple):
            out = out[0]
        # tf.nn.in_top_k (ties at the boundary count as correct), HIP kernel on the GPU
        c1 += int(E.in_top_k(out, y, 1).sum())
        c5 += int(E.in_top_k(out, y, min(5, out.shape[-1])).sum())
    total = num_iter * batch_size
    return c1 / total, c5 / total


def evaluate(preset, flags):
    F = flags.FLAGS
    cfg = trainer.PRESETS[preset]
    top5 = EVAL_DEFAULTS[preset][5]
    device = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    kw = {"resnet_size": F.resnet_size} if cfg["model"] == "cifar10_resnet_v2" else {}
    if cfg["model"].startswith("mobilenet") and "depth_multiplier" in F and F.depth_multiplier != 1.0:
        kw["depth_multiplier"] = F.depth_multiplier
    if "quantize" in F and F.quantize:  # create_eval_graph (mobilenet_v1_eval.py:126-127)
        from .compat.quantize import QuantConfig
        kw["quantize"] = QuantConfig(is_training=False)
    model = trainer.build_model_for_eval(preset, **kw).to(device)
    model.eval()
    if os.path.isdir(F.eval_dir):
        shutil.rmtree(F.eval_dir)
    os.makedirs(F.eval_dir, exist_ok=True)
    writer = SummaryWriter(F.eval_dir)
    data = _inputs(preset, flags, device)
    last = None
    n_evals = 0
    results = []
    while True:
        st = get_checkpoint_state(F.checkpoint_dir)  # re-read every poll
        path = st.model_checkpoint_path if st else None
        if not path:
            print("No checkpoint file found", flush=True)
        elif path != last:
            restore_for_eval(model, path, F.use_ema, prefix=cfg.get("scope_prefix", ""))
            gs = step_from_path(path)
            t0 = time.time()
            p1, r5 = eval_once(model, data, F.num_examples, F.batch_size, top5)
            dt = time.time() - t0
            if top5:
                print("%s: precision @ 1 = %.4f recall @ 5 = %.4f [%d examples] (%.1f examples/sec)"
                      % (datetime.now(), p1, r5, F.num_examples, F.num_examples / max(dt, 1e-9)), flush=True)
                writer.add_scalar("Recall @ 5", r5, gs)
            else:
                print("%s: precision @ 1 = %.3f, global_step: %d" % (datetime.now(), p1, gs), flush=True)
            writer.add_scalar("Precision @ 1", p1, gs)
            results.append((gs, p1, r5))
            last = path
            n_evals += 1
        if F.run_once or (F.max_evals and n_evals >= F.max_evals):
            break
        time.sleep(F.eval_interval_secs)
    writer.close()
    return results
