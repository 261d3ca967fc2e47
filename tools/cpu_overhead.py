#!/usr/bin/env python3
"""Host (CPU) enqueue time of an eager training step's phases vs the GPU step time: how far ahead of the GPU the
Python side runs.  No synchronisation inside the measured steps; the GPU time is a HIP-event bracket over the same
steps.  --force-comm: one rank over real RCCL (backend nccl, world 1) with every bucket all-reduce and the BN-statistics
sync issued (TrainStep(force_comm=True)): the host work a data-parallel rank adds per step, measured on one GPU.
Usage: python tools/cpu_overhead.py [--model resnet_v1_50] [--steps 10] [--force-comm] [--grad-comm bf16]"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet_v1_50")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--force-comm", action="store_true")
    ap.add_argument("--grad-comm", default="fp32", choices=("fp32", "bf16"))
    ap.add_argument("--graph", action="store_true", help="the captured step (with its collectives: graph_comm)")
    args = ap.parse_args()
    if args.force_comm:
        import socket

        import torch.distributed as dist
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=0, world_size=1)
    import bench
    from distributed_tensorflow_models_amd.engine import TrainStep
    from distributed_tensorflow_models_amd.models import nets_factory
    S, ncls, B, opt, extra = bench.PRESETS[args.model]
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    net = nets_factory.build(args.model, num_classes=ncls).to(dev)
    step = TrainStep(net, optimizer=opt, lr=0.1 if opt == "momentum" else 0.01, momentum=0.9, use_graph=args.graph,
                     force_comm=args.force_comm, graph_comm=args.graph,
                     grad_comm_dtype=torch.bfloat16 if args.grad_comm == "bf16" else None, **extra)
    x = torch.randn(B, S, S, 3, device=dev).to(torch.bfloat16)
    y = torch.randint(0, ncls, (B,), device=dev)
    marks = {}
    orig_fwd = step.model.forward
    orig_loss = step.loss_fn

    def fwd(*a, **k):
        t = time.perf_counter()
        out = orig_fwd(*a, **k)
        marks["fwd"] = marks.get("fwd", 0.0) + time.perf_counter() - t
        return out

    def loss_fn(*a, **k):
        t = time.perf_counter()
        out = orig_loss(*a, **k)
        marks["loss"] = marks.get("loss", 0.0) + time.perf_counter() - t
        marks["t_loss_end"] = time.perf_counter()
        return out
    for _ in range(5):
        step(x, y)
    torch.cuda.synchronize()
    step.model.forward, step.loss_fn = fwd, loss_fn
    marks["t_loss_end"] = 0.0  # (a replayed step runs no Python forward / loss: the phases stay 0)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    bwd = 0.0
    t0 = time.perf_counter()
    e0.record()
    for _ in range(args.steps):
        ts = time.perf_counter()
        step(x, y)
        if marks["t_loss_end"]:
            bwd += time.perf_counter() - marks["t_loss_end"]
    e1.record()
    host = time.perf_counter() - t0
    torch.cuda.synchronize()
    gpu = e0.elapsed_time(e1) / 1e3
    n = args.steps
    marks.setdefault("fwd", 0.0)
    marks.setdefault("loss", 0.0)
    print("%s%s%s: host enqueue per step %.2f ms (forward %.2f, loss %.2f, backward + optimizer %.2f); GPU per step %.2f "
          "ms; host / GPU %.0f %%%s" % (
              args.model, " [RCCL world 1, collectives forced, %s wire]" % args.grad_comm if args.force_comm else "",
              " [captured step]" if args.graph else "",
              host / n * 1e3, marks["fwd"] / n * 1e3, marks["loss"] / n * 1e3, bwd / n * 1e3, gpu / n * 1e3,
              100.0 * host / gpu, "; %d bucket all-reduces / step" % len(step.dp._done_works)
              if args.force_comm else ""), flush=True)
    step.dp.close()
    if args.force_comm:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
