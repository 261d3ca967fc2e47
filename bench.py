#!/usr/bin/env python3
"""Headline benchmark: ResNet-50 v1 (slim geometry) 224x224 bf16 training images/sec on MI355X.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N > 1 it is launched with
torch.distributed.run, one rank per GPU, RCCL over xGMI.  W untimed warmup steps, then exactly K
timed steps bracketed by barrier + device synchronize; the max wall time over ranks is used;
rank 0 prints ONE JSON line.  Weak scaling: the per-GPU batch is fixed as N grows.

Every timed step is a full training step: forward, softmax-xent loss, backward (hand-written HIP
conv/BN/pool kernels), bucketed RCCL all-reduce of all 25.6 M gradients (N > 1), and the fused
momentum-SGD + weight-decay update of every parameter.  Data: synthetic ImageNet-shaped batch
(random bf16 images, random labels) resident in HBM; weights random-init (no checkpoints/datasets).
"""
import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

BASELINE_VALUE = None  # the reference publishes no ResNet-50 images/sec
HEADLINE_METRIC = "images/sec (whole node) ResNet-50 224\u00d7224 bf16 at 1/2/4/8 MI355X"  # BASELINE.json

# BASELINE.json configs: model name -> (image size, classes, per-GPU batch, optimizer, extra TrainStep kwargs)
PRESETS = {
    "resnet_v1_50": (224, 1000, 256, "momentum", {}),
    # config #4: old-slim Inception-v3 as the reference trains it (RMSProp, label smoothing, aux head)
    "inception_v3_slim_old": (299, 1001, 128, "rmsprop", dict(label_smoothing=0.1, aux_weight=0.4, rho=0.9,
                                                              epsilon=1.0, wgrad_stream=False)),
    # config #5: VGG-16 with the reference's CIFAR geometry (10 classes, 134.3 M params)
    "vgg_16": (32, 10, 512, "sgd", {}),
    # config #1 plumbing model
    "lenet": (28, 10, 512, "sgd", {}),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=0, help="per-GPU batch (default: the preset's)")
    ap.add_argument("--model", default="resnet_v1_50", choices=sorted(PRESETS))
    ap.add_argument("--image-size", type=int, default=0)
    ap.add_argument("--bucket-mb", type=float, default=32.0)
    ap.add_argument("--grad-comm", default="fp32", choices=("fp32", "bf16"),
                    help="dtype of the gradient all-reduce on the wire (bf16 halves the xGMI bytes)")
    ap.add_argument("--wgrad-stream", type=int, default=-1,
                    help="weight gradients on the side stream: 1 / 0, -1 = the preset's choice")
    ap.add_argument("--graph", type=int, default=-1,
                    help="capture the step in a hipGraph (1/0); -1 = auto: on for launch-bound models on 1 GPU")
    ap.add_argument("--profile-steps", type=int, default=0)
    ap.add_argument("--dist-backend", default="", help="override the process-group backend (default: nccl = "
                    "RCCL on GPUs, gloo on CPU); gloo on GPUs lets several ranks share one device for rehearsals")
    ap.add_argument("--rccl-channels", type=int, default=0,
                    help="pin the RCCL channel count (NCCL_MIN/MAX_NCHANNELS); 0 = RCCL's own choice")
    ap.add_argument("--device", default="cuda", choices=("cuda", "cpu"),
                    help="cpu: the plumbing config (LeNet over gloo, no GPU; BASELINE.json config 1)")
    args = ap.parse_args()

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        # self-launch (mirrors reference train.sh:46-61, one process per worker): the parent never
        # touches the GPU; it starts N fresh ranks and forwards their output
        sys.exit(_launch_ranks(args.gpus))
    if env_world is not None and int(env_world) != args.gpus:
        print("bench.py: WORLD_SIZE=%s but --gpus %d; refusing to report a mismatched run" % (env_world, args.gpus),
              file=sys.stderr, flush=True)
        sys.exit(2)

    import torch
    import torch.distributed as dist

    world = int(env_world or "1")
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    cpu = args.device == "cpu"
    ndev = 0 if cpu else max(torch.cuda.device_count(), 1)
    gpu_index = local_rank % ndev if ndev else 0  # ranks > devices only in shared-GPU gloo rehearsals
    if world > 1:
        backend = args.dist_backend or ("gloo" if cpu else "nccl")
        if cpu or backend == "gloo":
            if not cpu:
                torch.cuda.set_device(gpu_index)
            dist.init_process_group("gloo")
        else:
            from distributed_tensorflow_models_amd.parallel import process_group as pg
            # per-bucket collective timing (read after the timed steps) + optional channel pinning
            pg.rccl_env(args.rccl_channels, timing=True)
            torch.cuda.set_device(local_rank)
            opts = pg.nccl_options(high_priority=True)  # comm stream ahead of queued backward kernels
            kw = {"pg_options": opts} if opts is not None else {}
            dist.init_process_group(backend, device_id=torch.device("cuda", local_rank), **kw)
    dev = torch.device("cpu") if cpu else torch.device("cuda", gpu_index)
    sync = (lambda: None) if cpu else torch.cuda.synchronize

    from distributed_tensorflow_models_amd.engine import TrainStep
    from distributed_tensorflow_models_amd.models import nets_factory

    if args.graph < 0:
        # measured on one MI355X (profiles/ab/r2_ab_graph_bench.log): LeNet 396k -> 875k img/s with the
        # captured step, Inception-v3 +0.5 % (885 launches per step), VGG-16 +0.2 %; ResNet-50 is
        # GPU-bound (+0.1 %, within noise) and stays eager
        args.graph = int(args.model in ("lenet", "inception_v3_slim_old", "vgg_16") and world == 1 and not cpu)
    # --graph 1 with several ranks: the step is captured WITH its RCCL bucket all-reduces and BN-statistics sync
    # (TrainStep graph_comm; bit-identical to eager at world 1, tests/test_distributed.py::
    # test_bsp_rccl_captured_step_matches_eager).  Opt-in: the auto policy keeps multi-rank steps eager.
    torch.manual_seed(1234)  # identical replicas: every rank builds the same initial weights
    S0, ncls, B0, opt, extra = PRESETS[args.model]
    if args.wgrad_stream >= 0:
        extra = dict(extra, wgrad_stream=bool(args.wgrad_stream))
    S = args.image_size or S0
    B = args.batch or B0
    kw = {"fc_conv_padding": "SAME"} if args.model == "vgg_16" else {}
    net = nets_factory.build(args.model, num_classes=ncls, **kw).to(dev)
    if world > 1:  # and make it explicit (the reference's chief-initialises-then-workers-wait contract)
        from distributed_tensorflow_models_amd.parallel import process_group as pg
        pg.broadcast_tensors(list(net.parameters()) + list(net.buffers()))
    torch.manual_seed(1234 + rank)  # each rank its own synthetic batch
    from distributed_tensorflow_models_amd.ops import elementwise as _ew
    _ew.set_base_seed(1234, rank)  # and its own dropout masks
    # one learning rate at every N (no linear x W scaling here, unlike the trainers' C16): the same
    # update math at 1..8 GPUs, and no early divergence of a random-init net at lr 0.8 on random labels
    step = TrainStep(net, optimizer=opt, lr=0.1 if opt == "momentum" else 0.01, momentum=0.9,
                     bucket_mb=args.bucket_mb, use_graph=bool(args.graph),
                     graph_comm=bool(args.graph) and world > 1,
                     grad_comm_dtype=torch.bfloat16 if args.grad_comm == "bf16" else None, **extra)
    cin = 1 if args.model == "lenet" else 3
    images = torch.randn(B, S, S, cin, device=dev).to(torch.float32 if cpu else torch.bfloat16)
    labels = torch.randint(0, ncls, (B,), device=dev)

    for _ in range(args.warmup):
        step(images, labels)
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step(images, labels)
    sync()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    phases = {}
    if world > 1 and not cpu and not args.graph:
        # after (outside) the timed region: 3 steps with HIP events on the compute stream.  The
        # "allreduce" section runs from the last backward kernel to the moment the compute stream
        # may proceed past every bucket's collective = the exposed (non-overlapped) all-reduce time.
        from distributed_tensorflow_models_amd.utils.metrics import StepTimer
        step.timer, acc = StepTimer(cuda=True), {}
        for _ in range(3):
            step(images, labels)
            for k, v in step.timer.sections().items():
                acc[k] = acc.get(k, 0.0) + v / 3
        step.timer = None
        t = torch.tensor([acc.get(k, 0.0) for k in ("fwd_ms", "bwd_ms", "allreduce_ms", "optimizer_ms")],
                         device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        phases = dict(zip(("fwd_ms", "bwd_ms", "allreduce_exposed_ms", "optimizer_ms"),
                          [round(float(v), 3) for v in t.tolist()]))
        bms = step.dp.bucket_ms()  # rank-local durations of each bucket's all-reduce, last step
        if bms:
            phases["bucket_allreduce_ms"] = bms
            phases["bucket_mb"] = [round(n * 4 / 1e6, 2) for n in step.dp.bucket_elements()]
    ms = dt / args.steps * 1000.0
    value = world * B * args.steps / dt
    if rank == 0:
        out = {
            "metric": HEADLINE_METRIC if args.model == "resnet_v1_50" else
            "images/sec (whole node) %s %dx%d %s training" % (args.model, S, S, "fp32 cpu" if cpu else "bf16"),
            "value": round(value, 2),
            "unit": "images/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": (round(value / BASELINE_VALUE, 4) if BASELINE_VALUE else None),
            "dtype": "fp32" if cpu else "bf16",
            "data": "synthetic (random %dx%dx%d %s images, random labels, random-init weights)" % (
                S, S, cin, "fp32" if cpu else "bf16"),
            "config": {"model": args.model, "global_batch": world * B, "per_gpu_batch": B, "seq_len": None,
                       "image_size": S, "parallelism": "dp%d" % world, "device": args.device,
                       "grad_allreduce_dtype": args.grad_comm,
                       # bytes each rank contributes to the gradient all-reduce per step (dead-tap windows
                       # excluded: parallel/bsp.py compact buckets)
                       "grad_wire_mb": round(step.dp.wire_elements() * (2 if args.grad_comm == "bf16" else 4) / 1e6,
                                             1),
                       # max over ranks, measured after the timed steps (N > 1 only)
                       "phases_ms": phases or None,
                       "optimizer": {"momentum": "momentum-sgd+wd", "rmsprop": "rmsprop(TF)+wd", "sgd": "sgd+wd"}[opt],
                       "final_loss": round(float(loss), 4) if math.isfinite(float(loss)) else None},
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def _launch_ranks(n):
    """Start ``n`` ranks of this script under torch.distributed.run (subprocess, never exec) and
    return the worst child exit code.  Rank 0's JSON line reaches stdout through the child."""
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC for RCCL on this host driver
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__)] + sys.argv[1:]
    proc = subprocess.Popen(cmd, env=env, start_new_session=True)
    try:
        return proc.wait()
    except KeyboardInterrupt:
        os.killpg(proc.pid, 15)
        return proc.wait()


if __name__ == "__main__":
    main()
