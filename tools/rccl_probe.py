#!/usr/bin/env python3
"""Step-by-step probe of the data-parallel path over RCCL on the GPUs of one box (one rank per GPU; with one GPU the
BSP collectives are forced on at world size 1).  Every stage prints before and after, so a hang names its stage.

  python tools/rccl_probe.py            (one rank; torchrun --nproc-per-node N tools/rccl_probe.py for N)"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def say(msg):
    print("[rank %s %.2fs] %s" % (os.environ.get("RANK", "0"), time.time() - T0, msg), flush=True)


T0 = time.time()


def main():
    import torch.distributed as dist

    from distributed_tensorflow_models_amd.parallel import process_group as pg
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29611")
    timing = os.environ.get("PROBE_TIMING", "1") == "1"
    pg.rccl_env(0, timing=timing)
    say("init nccl (timing %s, high-priority %s)" % (timing, os.environ.get("PROBE_HIPRIO", "1")))
    pg.init(backend="nccl", timeout_s=60, force=True, high_priority=os.environ.get("PROBE_HIPRIO", "1") == "1")
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
    W = dist.get_world_size()
    say("initialised: world %d" % W)
    t = torch.ones(1 << 20, device=dev)
    dist.all_reduce(t)
    torch.cuda.synchronize()
    say("sync all_reduce ok (%.0f)" % float(t[0]))
    w = dist.all_reduce(t, async_op=True)
    w.wait()
    torch.cuda.synchronize()
    say("async all_reduce + wait ok")
    side = torch.cuda.Stream(device=dev)
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        w = dist.all_reduce(t, async_op=True)
    w.wait()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    say("all_reduce issued from a side stream ok")
    if timing:
        say("duration of the last collective: %.4f ms" % float(w._get_duration()))
    from distributed_tensorflow_models_amd.engine import TrainStep
    from distributed_tensorflow_models_amd.models import nets_factory
    torch.manual_seed(0)
    model = nets_factory.build(os.environ.get("PROBE_MODEL", "resnet_v1_50"), num_classes=16).to(dev)
    step = TrainStep(model, optimizer="momentum", lr=0.05, momentum=0.9, bucket_mb=2.0, force_comm=True)
    say("TrainStep built: %d buckets, BN flat %d" % (len(step.dp.buckets), step.bufsync.numel()))
    g = torch.Generator().manual_seed(5)
    x = torch.randn(8, 64, 64, 3, generator=g).to(dev, torch.bfloat16)
    y = torch.randint(0, 16, (8,), generator=g).to(dev)
    for i in range(3):
        say("step %d: forward/backward" % i)
        loss, _skip = step._forward_backward(x, y)
        say("step %d: backward issued (%d collectives in flight)" % (i, len(step.dp._done_works)))
        step.opt.step(0.05, grad_scale=step.dp.grad_scale, skip_flag=_skip)
        torch.cuda.synchronize()
        say("step %d: done, loss %.4f" % (i, float(loss)))
    if timing:
        say("bucket durations: %s" % step.dp.bucket_ms()[:4])
    step.dp.close()
    dist.destroy_process_group()
    say("ok")


if __name__ == "__main__":
    main()
