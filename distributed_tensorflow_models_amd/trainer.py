"""Generic distributed trainer behind every reference entry script.

One process per MI355X.  ``train(preset, FLAGS)`` reproduces the reference trainer skeleton with
MI355X-native machinery underneath:
  parse flags -> (ps: no-op join) -> process group (torchrun env or --ps_hosts/--worker_hosts)
  -> model (TF names) -> input pipeline -> loss/optimizer/schedule (TF semantics)
  -> BSP (bucketed RCCL all-reduce) | ASP (owner-sharded store) | SSP (store + staleness clock)
  -> Supervisor (chief restore-or-init, periodic TF-layout checkpoints) -> step loop with the
  reference per-step log line, NaN guard, optional traces and JSONL metrics.
Deliberate fixes of reference defects: train_dir is NOT wiped unless --fresh,
BN moving statistics are always updated, chief-only duties stay on rank 0, VGG saves checkpoints.
"""
import math
import os
import shutil
import time

import numpy as np
import torch

from .ckpt.saver import Saver, TFVar, model_variables
from .compat import logging
from .compat.train import ExponentialDecay, Server
from .engine import TrainStep
from .models import nets_factory
from .parallel import process_group as pg
from .utils.heartbeat import Heartbeat
from .utils.metrics import JsonlMetrics, StepTimer, format_step
from .utils.profiler import StepTracer

CIFAR_TRAIN = 50000
IMAGENET_TRAIN = 1281167

# reference hyper-parameters per trainer (constants quoted from the reference trainer files)
PRESETS = {
    # cnn/cifar10_cnn_bsp.py:9-13,46-64 + cnn/cifar10.py:54-81
    "cnn": dict(model="cifar10_cnn", num_classes=10, dataset="cifar10", image_size=24, batch_size=512, lr=0.32,
                lr_scale_workers=False, decay_epochs=350.0, decay_factor=0.1, optimizer="sgd", ema=0.9999,
                wd_all=None, max_steps=20000, save_secs=60, log_style="cnn", max_to_keep=5,
                global_step_name="Variable",
                train_dir="/home/ubuntu/cifar10/train", data_dir="/home/ubuntu/cifar10/data"),
    # alexnet/cifar10_alexnet_bsp.py:18-30,54-94
    "alexnet": dict(model="alexnet_v2", num_classes=10, dataset="cifar10", image_size=32, batch_size=128, lr=0.01,
                    lr_scale_workers=True, decay_epochs=350.0, decay_factor=0.1, optimizer="sgd", ema=0.9999,
                    wd_all=2e-4, max_steps=2000000, save_secs=60, log_style="standard", max_to_keep=5,
                    scope_prefix="partitioned_space/", partitioned=True,
                    global_step_name="partitioned_space/Variable",
                    train_dir="/home/ubuntu/cifar10/train", data_dir="/home/ubuntu/cifar10/data"),
    # vgg/cifar10_vgg_bsp.py:19-30,57-95 (factory vgg_16, 10 classes, is_training=False -> no dropout)
    "vgg": dict(model="vgg_16", num_classes=10, dataset="cifar10", image_size=32, batch_size=72, lr=0.01,
                lr_scale_workers=True, decay_epochs=350.0, decay_factor=0.1, optimizer="sgd", ema=None,
                wd_all=2e-4, max_steps=20000, save_secs=60, log_style="standard", max_to_keep=5,
                model_kw=dict(fc_conv_padding="SAME", dropout_keep_prob=1.0, weight_decay=0.0),
                scope_prefix="root/", partitioned=True, global_step_name="root/Variable",
                train_dir="/home/ubuntu/cifar10_train", data_dir="/home/ubuntu/cifar10_data"),
    # vgg/cifar10_vgg_asp.py:20-31 + vgg/cifar10.py:338-391 (lr not scaled, var EMA)
    "vgg_asp": dict(model="vgg_16", num_classes=10, dataset="cifar10", image_size=32, batch_size=72, lr=0.01,
                    lr_scale_workers=False, decay_epochs=350.0, decay_factor=0.1, optimizer="sgd", ema=0.9999,
                    wd_all=2e-4, max_steps=20000, save_secs=60, log_style="standard", max_to_keep=5,
                    model_kw=dict(fc_conv_padding="SAME", dropout_keep_prob=1.0, weight_decay=0.0),
                    scope_prefix="root/", partitioned=True, global_step_name="root/Variable",
                    train_dir="/home/ubuntu/cifar10_train", data_dir="/home/ubuntu/cifar10_data"),
    # resnet/cifar10_resnet_bsp.py:19-29,57-106 (CIFAR ResNet v2, resnet_size 32)
    "resnet": dict(model="cifar10_resnet_v2", num_classes=10, dataset="cifar10", image_size=32, batch_size=128,
                   lr=0.08, lr_scale_workers=True, decay_epochs=32.0, decay_factor=0.1, optimizer="sgd",
                   ema=0.9999, wd_all=2e-3, max_steps=10000000, save_secs=60, log_style="short", max_to_keep=1,
                   # tf.layers.batch_normalization (resnet_model.py:45) keeps its moving statistics out of
                   # tf.moving_average_variables(): the EMA covers trainables only
                   ema_buffers=False,
                   train_accuracy_every=200, scope_prefix="root/", partitioned=True, global_step_name="Variable",
                   train_dir="/home/ubuntu/cifar10/train",
                   data_dir="/home/ubuntu/cifar10/data"),
    # cifarnet/cifar10_cifarnet_bsp.py:20-32,56-91
    "cifarnet": dict(model="cifarnet", num_classes=10, dataset="cifar10", image_size=32, batch_size=512, lr=0.1,
                     lr_scale_workers=True, decay_epochs=20.0, decay_factor=0.1, optimizer="sgd", ema=0.9999,
                     wd_all=2e-4, max_steps=2000000, save_secs=60, log_style="standard", max_to_keep=5,
                     scope_prefix="partitioned_space/", partitioned=True,
                     global_step_name="partitioned_space/Variable",
                     train_dir="/home/ubuntu/cifar10/train", data_dir="/home/ubuntu/cifar10/data"),
    # inception/imagenet_inception_bsp.py:54-72,104-157 (old-slim Inception-v3, RMSProp, label smoothing)
    "inception": dict(model="inception_v3_slim_old", num_classes=1001, dataset="imagenet", image_size=299,
                      batch_size=32, lr=0.045, lr_scale_workers=True, decay_epochs=2.0, decay_factor=0.94,
                      decay_div_workers=True, optimizer="rmsprop", rmsprop_decay=0.9, momentum=0.9,
                      rmsprop_epsilon=1.0, ema=0.9999, wd_all=None, label_smoothing=0.1, aux_weight=0.4,
                      max_steps=10000000, save_secs=600, log_style="short", max_to_keep=5, nan_guard=True,
                      train_dir="/home/ubuntu/imagenet/train/", data_dir="/home/ubuntu/imagenet/data/",
                      wipe=False, wgrad_stream=False),
    # vgg/nets/mobilenet_v1_train.py:57-160 (SGD 0.045, x0.94 every 2.5 epochs, batch 64)
    "mobilenet_v1": dict(model="mobilenet_v1", num_classes=1001, dataset="imagenet", image_size=224, batch_size=64,
                         lr=0.045, lr_scale_workers=False, decay_epochs=2.5, decay_factor=0.94, optimizer="sgd",
                         ema=None, wd_all=None, max_steps=10000000, save_secs=100,
                         log_style="short", max_to_keep=5, train_dir="/tmp/mobilenet_v1_train",
                         data_dir="/tmp/imagenet"),
    # headline benchmark model (north star) - slim resnet_v1_50 on synthetic ImageNet
    "resnet50": dict(model="resnet_v1_50", num_classes=1000, dataset="synthetic_imagenet", image_size=224,
                     batch_size=256, lr=0.1, lr_scale_workers=True, decay_epochs=30.0, decay_factor=0.1,
                     optimizer="momentum", momentum=0.9, ema=None, wd_all=None, max_steps=1000, save_secs=600,
                     log_style="standard", max_to_keep=5, train_dir="/tmp/resnet50_train", data_dir=""),
    # BASELINE config #1 plumbing: LeNet on synthetic MNIST
    "lenet": dict(model="lenet", num_classes=10, dataset="synthetic_mnist", image_size=28, batch_size=64, lr=0.01,
                  lr_scale_workers=True, decay_epochs=100.0, decay_factor=0.1, optimizer="sgd", ema=None,
                  wd_all=None, max_steps=200, save_secs=60, log_style="standard", max_to_keep=5,
                  train_dir="/tmp/lenet_train", data_dir=""),
}


def define_common_flags(flags, preset):
    """Flags shared by every trainer (reference flag inventory) + MI355X extras."""
    p = PRESETS[preset]
    d = flags.DEFINE_string, flags.DEFINE_integer, flags.DEFINE_float, flags.DEFINE_boolean
    S, I, Fl, B = d
    for name, fn, default, h in (
            ("job_name", S, "", "One of 'ps', 'worker'"),
            ("ps_hosts", S, "", "Comma-separated list of hostname:port pairs"),
            ("worker_hosts", S, "", "Comma-separated list of hostname:port pairs"),
            ("task_id", I, 0, "Task id of the replica running the training."),
            ("batch_size", I, p["batch_size"], "Number of images to process in a batch."),
            ("data_dir", S, p["data_dir"], "Path to the data directory."),
            ("train_dir", S, p["train_dir"], "Directory where to write event logs and checkpoint."),
            ("max_steps", I, p["max_steps"], "Number of batches to run."),
            ("log_device_placement", B, preset == "cnn", "Whether to log device placement."),
            ("resnet_size", I, 32, "The size of the ResNet model to use."),
            ("protocol", S, "grpc", "accepted for compatibility; transport is RCCL/gloo"),
            ("save_interval_secs", I, p["save_secs"], "Save interval seconds."),
            ("save_every_steps", I, 0, "also checkpoint every N global steps (0 = time-based only)"),
            ("save_summaries_secs", I, 180, "train-side TensorBoard scalars at most this often (0 = off)"),
            ("initial_learning_rate", Fl, p["lr"], "Initial learning rate."),
            ("num_epochs_per_decay", Fl, p["decay_epochs"], "Epochs after which learning rate decays."),
            ("learning_rate_decay_factor", Fl, p["decay_factor"], "Learning rate decay factor."),
            # MI355X-native extras
            ("sync_mode", S, "", "bsp | asp | ssp (default from the entry script)"),
            ("max_staleness", I, 5, "SSP staleness bound in local steps"),
            ("synthetic_data", B, False, "use HBM-resident synthetic batches"),
            ("bucket_mb", Fl, 32.0, "all-reduce bucket size (MB)"),
            ("use_hipgraph", B, False, "capture the BSP training step in a hipGraph (launch-bound models; "
             "single-rank only, ignored with a warning when world > 1)"),
            ("bn_sync_every", I, 1, "BSP: average the BN moving statistics over the replicas every N steps"),
            ("rccl_channels", I, 0, "pin the RCCL channel count (0 = RCCL's choice)"),
            ("grad_comm_dtype", S, "fp32", "gradient all-reduce dtype on the wire: fp32 | bf16"),
            ("deterministic", B, False, "bit-reproducible GPU reductions (no cross-block fp32 atomics)"),
            ("trace_steps", S, "", "a:b -> export a Chrome trace of steps [a, b)"),
            ("fresh", B, False, "wipe train_dir before training (the reference always did)"),
            ("log_every", I, 1, "log the per-step line every N steps"),
            ("metrics_file", S, "", "JSONL metrics path (rank 0)"),
            ("batch_weight", Fl, 1.0, "per-rank gradient weight b_r/b_nominal (C15)"),
            ("fault_inject", S, "", "rank:step[:hang] -> hard-exit (or hang) that rank at that step (resume tests)"),
            ("seed", I, 0, "random seed"),
            ("depth_multiplier", Fl, 1.0, "MobileNet depth multiplier"),
            ("fine_tune_checkpoint", S, "", "initialise model variables from this checkpoint (fresh runs only)"),
            ("train_accuracy_every", I, p.get("train_accuracy_every", 0),
             "every worker: every N steps, accuracy of the training-mode network on a fed batch of distorted training "
             "images (reference resnet/cifar10_resnet_bsp.py:146-148; 0 = off)"),
            ("train_accuracy_batch", I, 10000, "images in that fed batch (the reference feeds 10000)"),
    ):
        fn(name, default, h)
        flags.FLAGS.reset(name)  # the entry script's preset defaults win


def _device():
    if torch.cuda.is_available():
        return torch.device("cuda", int(os.environ.get("LOCAL_RANK", 0)))
    return torch.device("cpu")


def make_input(cfg, batch_size, device, flags, rank):
    ds = "synthetic_imagenet" if flags.synthetic_data and cfg["dataset"] == "imagenet" else cfg["dataset"]
    S = cfg["image_size"]
    if ds == "cifar10":
        from .data import cifar10
        return cifar10.distorted_inputs(flags.data_dir, batch_size, S, device=device, seed=flags.seed + rank)
    if ds == "synthetic_mnist":
        from .data.synthetic import synthetic_mnist

        class _M:
            def __init__(self):
                self.x, self.y = synthetic_mnist(batch_size * 16, device, flags.seed + rank)
                self.i = 0

            def next_batch(self):
                s = (self.i % 16) * batch_size
                self.i += 1
                return self.x[s:s + batch_size], self.y[s:s + batch_size]
        return _M()
    if ds == "imagenet":
        from .data import imagenet
        if torch.device(device).type == "cuda":
            # decode on host threads, crop / resize / flip / colour on the GPU (data/imagenet_gpu.py); the node's
            # host CPUs are checked against what its ranks consume (data/capacity.py), and the device JPEG decode
            # (host marker parse only; HIP Huffman / IDCT / colour) is chosen when the full host decode cannot keep up
            from .data import capacity, imagenet_gpu
            split = capacity.choose_split_decode(cfg["model"])
            capacity.decode_capacity_check(cfg["model"], mode=split, log=logging.warning)
            return imagenet_gpu.distorted_inputs(imagenet.ImagenetData("train", flags.data_dir), batch_size,
                                                 image_size=S, device=device, seed=flags.seed + rank,
                                                 split_decode=split)
        return imagenet.distorted_inputs(imagenet.ImagenetData("train", flags.data_dir), batch_size, image_size=S,
                                         device=device, seed=flags.seed + rank)
    from .data.synthetic import SyntheticImages
    return SyntheticImages(batch_size, S, S, 3, cfg["num_classes"], device, seed=flags.seed + rank,
                           label_offset=1 if cfg["num_classes"] == 1001 else 0)


def make_loss_fn(label_smoothing=0.0, aux_weight=0.4, batch_weight=1.0):
    """Cross-entropy (+ weighted aux head) on the HIP softmax-xent kernel; L2 terms are applied as
    coupled weight decay inside the optimizer (identical gradient, K14)."""
    from .ops import nn as F

    def loss_fn(out, labels):
        aux = None
        if isinstance(out, tuple):
            out, aux = out
        heads = [(out, batch_weight)]
        if aux is not None and aux_weight:
            heads.append((aux, aux_weight * batch_weight))
        return F.mean_xent_loss(heads, labels, label_smoothing)
    return loss_fn


def train(preset, flags, default_mode="bsp"):
    FLAGS = flags.FLAGS
    cfg = dict(PRESETS[preset])
    mode = (FLAGS.sync_mode or default_mode).lower()
    logging.set_verbosity(logging.INFO)
    ps_hosts = [h for h in FLAGS.ps_hosts.split(",") if h]
    worker_hosts = [h for h in FLAGS.worker_hosts.split(",") if h]
    if FLAGS.job_name == "ps":
        Server({"ps": ps_hosts, "worker": worker_hosts}, "ps", FLAGS.task_id).join()
        return 0
    # RCCL knobs before the communicator exists: channel count, per-bucket timing for the JSONL metrics
    pg.rccl_env(FLAGS.rccl_channels, timing=bool(FLAGS.metrics_file))
    if worker_hosts and "WORLD_SIZE" not in os.environ:
        Server({"ps": ps_hosts, "worker": worker_hosts}, "worker", FLAGS.task_id)
    else:
        pg.init()
    rank, world = pg.rank(), pg.world_size()
    device = _device()
    logging.info("replica %d of world %d (%s, %s)", rank, world, mode, device)
    torch.manual_seed(FLAGS.seed + (rank if mode != "bsp" else 0))
    from .ops import elementwise as _ew
    _ew.set_base_seed(FLAGS.seed, rank)  # independent dropout masks per replica
    if FLAGS.deterministic and device.type == "cuda":
        from .ops import _lib
        _lib.set_deterministic(True)

    # ---- model ---------------------------------------------------------------------------------
    mkw = dict(cfg.get("model_kw", {}))
    if cfg["model"] == "cifar10_resnet_v2":
        mkw["resnet_size"] = FLAGS.resnet_size
    if cfg["model"].startswith("mobilenet") and FLAGS.depth_multiplier != 1.0:
        mkw["depth_multiplier"] = FLAGS.depth_multiplier
    if "quantize" in FLAGS and FLAGS.quantize:
        # tf.contrib.quantize.create_training_graph(quant_delay=get_quant_delay())
        # (reference vgg/nets/mobilenet_v1_train.py:66-73,138-139): quantise at once when fine-tuning
        from .compat.quantize import QuantConfig
        mkw["quantize"] = QuantConfig(quant_delay=0 if FLAGS.fine_tune_checkpoint else FLAGS.quant_delay)
    model = nets_factory.build(cfg["model"], num_classes=cfg["num_classes"], **mkw).to(device)
    if cfg.get("wd_all") is not None:  # loss += wd * sum(l2_loss(v) for v in trainable_variables())
        for p in model.parameters():
            if p.requires_grad:
                p.weight_decay = cfg["wd_all"]
    B = FLAGS.batch_size
    data = make_input(cfg, B, device, FLAGS, rank)

    # ---- schedule (C16, C19) ---------------------------------------------------------------------
    n_train = CIFAR_TRAIN if cfg["dataset"] in ("cifar10",) else IMAGENET_TRAIN
    batches_per_epoch = n_train / float(B)
    decay_steps = batches_per_epoch * FLAGS.num_epochs_per_decay
    if cfg.get("decay_div_workers") and mode == "bsp":
        decay_steps /= max(world, 1)
    scale = world if (cfg["lr_scale_workers"] and mode == "bsp") else 1
    sched = ExponentialDecay(FLAGS.initial_learning_rate * scale, max(decay_steps, 1.0),
                             FLAGS.learning_rate_decay_factor, staircase=True)
    opt_kw = dict(optimizer=cfg["optimizer"], lr=sched(0), momentum=cfg.get("momentum", 0.9),
                  rho=cfg.get("rmsprop_decay", 0.9), epsilon=cfg.get("rmsprop_epsilon", 1e-10))

    # ---- engine + supervisor / checkpoints (C7, §5.4) -------------------------------------------
    from .compat.train import Supervisor, latest_checkpoint
    is_chief = rank == 0
    if is_chief and FLAGS.fresh and os.path.isdir(FLAGS.train_dir):
        shutil.rmtree(FLAGS.train_dir)
    pg.barrier()
    path = latest_checkpoint(FLAGS.train_dir) if os.path.isdir(FLAGS.train_dir) else None
    # TF variable layout of the trainer: its variable_scope prefix and, for the
    # partitioned scopes, P = len(ps_hosts) axis-0 slices per variable (tf.fixed_size_partitioner)
    ckpt_kw = dict(prefix=cfg.get("scope_prefix", ""),
                   partitions=max(1, len(ps_hosts)) if cfg.get("partitioned") else None)
    gstep = torch.zeros((), dtype=torch.int64)
    loss_fn = make_loss_fn(cfg.get("label_smoothing", 0.0), cfg.get("aux_weight", 0.4), FLAGS.batch_weight)
    store = clock = None
    ft_missing = None
    if FLAGS.fine_tune_checkpoint and not path:
        # model variables only (no slots, no global step: the schedule restarts), missing ones keep their
        # initialisation (e.g. a new logits layer).  Restored BEFORE the engine / store exist, so the BSP
        # broadcast, the BN-statistics sync snapshot, the bf16 compute copies and the ASP owner shards all start
        # from the fine-tune values (a restore after them would be folded into the next BN sync as a W-fold delta)
        ft = [v for v in model_variables(model, None, None, prefix=ckpt_kw["prefix"])]
        ft_missing = Saver(ft).restore(FLAGS.fine_tune_checkpoint, strict=False)
    if mode == "bsp":
        if FLAGS.use_hipgraph and world > 1:
            logging.warning("--use_hipgraph ignored: step capture is single-rank only (world size %d)", world)
        step_fn = TrainStep(model, bucket_mb=FLAGS.bucket_mb, label_smoothing=cfg.get("label_smoothing", 0.0),
                            aux_weight=cfg.get("aux_weight", 0.4), ema_decay=cfg.get("ema"), lr_schedule=sched,
                            batch_weight=FLAGS.batch_weight, use_graph=FLAGS.use_hipgraph and world == 1,
                            ema_buffers=cfg.get("ema_buffers", True), bn_sync_every=FLAGS.bn_sync_every,
                            wgrad_stream=cfg.get("wgrad_stream"),
                            grad_comm_dtype=torch.bfloat16 if FLAGS.grad_comm_dtype == "bf16" else None,
                            timer=StepTimer() if (FLAGS.metrics_file and rank == 0 and not FLAGS.use_hipgraph)
                            else None, **opt_kw)
        vars_ = model_variables(model, step_fn.opt, gstep, **ckpt_kw)
        vars_[-1].name = cfg.get("global_step_name", "global_step")
        if path:
            Saver(vars_).restore(path)
        if world > 1:  # one collective replaces the reference's chief-init + 1 s polling of workers
            pg.broadcast_tensors([v.tensor for v in vars_ if v.tensor.is_floating_point()] +
                                 [b for b in model.buffers()])
        from .ops.nn import invalidate_weight_copies
        invalidate_weight_copies(model.parameters())  # bf16 compute copies follow the restored weights
        step_fn.bufsync.resync()  # the BN statistics' sync snapshot follows the restored / broadcast values
        step_fn.global_step = int(gstep)
        step_fn.opt.num_updates = int(gstep)
    elif mode in ("asp", "ssp"):
        from .engine import moving_average_buffers, prepare_compute_copies
        from .parallel.asp import ASPTrainStep, ParamStore
        from .parallel.ssp import StalenessClock
        vars_ = model_variables(model, None, gstep, **ckpt_kw)
        vars_[-1].name = cfg.get("global_step_name", "global_step")
        if path:  # owners initialise their shards from the restored replica
            Saver(vars_).restore(path)
        prepare_compute_copies(model)
        store = ParamStore(list(model.parameters()), cfg["optimizer"], sched(0), opt_kw["momentum"], opt_kw["rho"],
                           opt_kw["epsilon"], run_id=os.environ.get("DTM_RUN_ID", "0"),
                           buffers=moving_average_buffers(model))
        if is_chief and int(gstep):
            store.set_global_step(int(gstep))
        # optimizer slots live in the owner shards: checkpointed from there, restored into them
        slot_vars = [v for v in model_variables(model, None, None, store=store, **ckpt_kw)
                     if v.name.endswith(("/Momentum", "/RMSProp", "/RMSProp_1"))]
        if path and is_chief and slot_vars:
            Saver(slot_vars).restore(path, strict=False)
        vars_ = vars_[:-1] + slot_vars + vars_[-1:]
        pg.barrier()
        if mode == "ssp":
            clock = StalenessClock(FLAGS.max_staleness, log_fn=logging.info)
        step_fn = ASPTrainStep(model, loss_fn, store, sched, clock)
    else:
        raise ValueError("sync_mode must be bsp, asp or ssp")
    if path:
        logging.info("rank %d restored %s (global_step %d)", rank, path, int(gstep))
    elif FLAGS.fine_tune_checkpoint:
        logging.info("fine-tuning from %s (%d variables not in the checkpoint)", FLAGS.fine_tune_checkpoint,
                     len(ft_missing or []))
    saver = Saver(vars_, max_to_keep=cfg["max_to_keep"])
    if is_chief and os.path.isdir(FLAGS.train_dir):
        saver.recover_last_checkpoints(FLAGS.train_dir)
    sv = Supervisor(is_chief=is_chief, logdir=FLAGS.train_dir, saver=saver, global_step=gstep,
                    save_model_secs=FLAGS.save_interval_secs)
    start = int(gstep) if mode == "bsp" else store.global_step() if is_chief else int(gstep)

    metrics = JsonlMetrics(FLAGS.metrics_file if is_chief else None)
    tracer = StepTracer(FLAGS.trace_steps, os.path.join(FLAGS.train_dir, "traces"), rank)
    fault = None
    if FLAGS.fault_inject and os.environ.get("DTM_ATTEMPT", "0") == "0":  # only the first attempt
        parts = FLAGS.fault_inject.split(":")
        fault = (int(parts[0]), int(parts[1]), parts[2] if len(parts) > 2 else "exit")
    heartbeat = Heartbeat(rank)

    # training-side TensorBoard scalars (the graph-side summaries the reference defines, e.g.
    # cnn/cifar10.py:309-335,361: learning_rate, total_loss (raw) and its 0.9 moving average), written
    # to train_dir by the chief at most every --save_summaries_secs
    from .utils.tb import SummaryWriter
    tbw = SummaryWriter(FLAGS.train_dir) if (is_chief and FLAGS.save_summaries_secs > 0) else None
    loss_avg, t_summary = None, None

    # ---- loop (reference hot loop) ------------------------------------------------
    step = start if mode == "bsp" else 0
    probe = None  # the --train_accuracy_every input pipeline (created on first use)
    loss_v = float("nan")
    t_log, n_since = time.time(), 0
    while step < FLAGS.max_steps:
        if fault and fault[0] == rank and fault[1] == step:
            if fault[2] == "hang":
                logging.error("fault injection: rank %d hangs at step %d", rank, step)
                while True:  # a wedged rank: alive, silent, never reaches the next collective
                    time.sleep(3600)
            logging.error("fault injection: rank %d exits at step %d", rank, step)
            os._exit(17)
        tracer.step(step)
        images, labels = data.next_batch()
        if mode == "bsp":
            loss = step_fn(images, labels)
            gs = step_fn.global_step
        else:
            loss, gs = step_fn(images, labels)
        n_since += 1
        log_now = step % max(FLAGS.log_every, 1) == 0 or step + 1 >= FLAGS.max_steps
        # the loss is read (a device sync) on log steps only; the NaN assertion of the reference
        # (imagenet_inception_bsp.py:191, every step) is checked there, and non-finite steps in
        # between are caught by the engine's device-side guard (update skipped, counted, reported)
        need_log = log_now
        if need_log:
            loss_v = float(loss)
        dt = 0.0
        if log_now:
            # the device is drained only on logged steps (the time is averaged over the steps since the
            # last log line); the other steps leave the host free to run ahead of the GPU
            if device.type == "cuda":
                torch.cuda.synchronize()
            now = time.time()
            dt = (now - t_log) / n_since
            t_log, n_since = now, 0
        if cfg.get("nan_guard") and math.isnan(loss_v):  # imagenet_inception_bsp.py:191
            raise FloatingPointError("Model diverged with loss = NaN")
        if mode == "bsp" and need_log and step_fn.poll_skipped():
            if cfg.get("nan_guard"):
                # the reference asserts on a NaN loss every step; here the device-side guard skipped the update
                # of a non-finite step and the check fires at the next log line (at most --log_every steps late)
                raise FloatingPointError("Model diverged with loss = NaN (non-finite gradients at a step since "
                                         "the last log line; %d update(s) skipped)" % step_fn.skipped)
            logging.warning("step %d: non-finite gradients since the last log line, update(s) skipped (%d so far)",
                            step, step_fn.skipped)
        gstep.fill_(gs)
        if log_now:
            print(format_step(cfg["log_style"], step, gs, loss_v, B / max(dt, 1e-9), dt), flush=True)
            if tbw is not None and loss_v == loss_v:
                loss_avg = loss_v if loss_avg is None else 0.9 * loss_avg + 0.1 * loss_v
                if t_summary is None or time.time() - t_summary >= FLAGS.save_summaries_secs:
                    t_summary = time.time()
                    tbw.add_scalar("learning_rate", float(sched(gs)), gs)
                    tbw.add_scalar("total_loss (raw)", loss_v, gs)
                    tbw.add_scalar("total_loss", loss_avg, gs)
                    tbw.add_scalar("images_per_sec", world * B / max(dt, 1e-9), gs)
            extra = step_fn.timer.sections() if (mode == "bsp" and step_fn.timer is not None) else {}
            if mode == "bsp" and metrics.f is not None and world > 1:
                bms = step_fn.dp.bucket_ms()  # per-bucket all-reduce durations (RCCL timing events)
                if bms:
                    extra["bucket_allreduce_ms"] = bms
            if device.type == "cuda" and metrics.f is not None:
                extra["max_mem_gb"] = torch.cuda.max_memory_allocated(device) / 2 ** 30
            metrics.write(step=step, global_step=gs, loss=loss_v, lr=sched(gs), images_per_sec=B / max(dt, 1e-9),
                          node_images_per_sec=world * B / max(dt, 1e-9), step_ms=dt * 1e3, world=world, mode=mode,
                          **extra)
        # every worker runs the probe, as every reference worker does (resnet/cifar10_resnet_bsp.py:146-148)
        if FLAGS.train_accuracy_every and step % FLAGS.train_accuracy_every == 0:
            if probe is None:
                probe = make_input(cfg, FLAGS.train_accuracy_batch, device, FLAGS, rank + 7919)
            acc = train_accuracy_probe(model, probe)
            # tf.logging.info('evaluation: step - '+str(step)+'; accuracy: '+ str(accuracy))
            logging.info("evaluation: step - %d; accuracy: %s", step, str(np.float32(acc)))
        if mode == "bsp" or is_chief:
            sv.maybe_save(gs, force=bool(FLAGS.save_every_steps) and gs % FLAGS.save_every_steps == 0)
        heartbeat.beat(step)
        step += 1
    if mode in ("asp", "ssp"):
        if clock is not None:
            clock.finish()
        store.pull()
    sv.maybe_save(int(gstep), force=True)
    metrics.close()
    if tbw is not None:
        tbw.close()
    if store is not None:  # owners keep their shards alive until every worker is done with them
        from .parallel.asp import wait_all_done
        wait_all_done(store.store, world, store.run_id)
        store.close()
    pg.barrier()
    return 0


def train_accuracy_probe(model, data):
    """The reference's training-set accuracy probe (resnet/cifar10_resnet_bsp.py:66-70,146-148): accuracy_op =
    mean(argmax(network(inputs, True)) == labels) run on one fed batch of distorted training images - the
    network in TRAINING mode (batch statistics), whose BN moving averages that sess.run leaves alone (the
    reference never runs UPDATE_OPS there).  Here the moving statistics are saved and restored around the
    forward (the fused training-mode kernels update them in place)."""
    from .engine import moving_average_buffers
    bufs = moving_average_buffers(model)
    saved = [b.detach().clone() for b in bufs]
    images, labels = data.next_batch()
    with torch.no_grad():
        out = model(images, training=True)
        if isinstance(out, tuple):
            out = out[0]
        from .ops.lazy import as_tensor
        acc = (as_tensor(out).float().argmax(-1) == labels).float().mean().item()
        for b, v in zip(bufs, saved):
            b.copy_(v)
    return acc


def build_model_for_eval(preset, flags_values=None, **kw):
    cfg = PRESETS[preset]
    mkw = dict(cfg.get("model_kw", {}))
    mkw.update(kw)
    return nets_factory.build(cfg["model"], num_classes=cfg["num_classes"], **mkw)


__all__ = ["PRESETS", "define_common_flags", "train", "TFVar"]
