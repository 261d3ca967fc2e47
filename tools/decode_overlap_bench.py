#!/usr/bin/env python3
"""What the device JPEG decode costs the training step it feeds: ResNet-50 224^2 batch-256 momentum steps (the bench.py
configuration) with, each step, the next batch's decode of 256 ImageNet-like JPEGs (tools/decode_cpu_cost.py
generator, ~70 KB) launched on a side stream - entropy decode (jpeg_huff_kernel) + IDCT / colour - against the same
steps without it.  Blocks of steps alternate (off / on / off / ...) so clock drift cancels.  The decode's stand-alone
time is printed too: a latency-bound decode co-running with the conv kernels costs the step far less than its own
duration.

Usage: python tools/decode_overlap_bench.py [--blocks 4] [--steps 10] [--cfg 256x11]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=4)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--cfg", default="256x11")
    ap.add_argument("--low-priority", type=int, default=0, help="decode stream at the least priority HIP allows")
    a = ap.parse_args()
    import torch

    from distributed_tensorflow_models_amd.data import jpeg
    from distributed_tensorflow_models_amd.engine import TrainStep
    from distributed_tensorflow_models_amd.models import nets_factory
    from distributed_tensorflow_models_amd.ops import _lib
    from tools.decode_cpu_cost import make_jpegs
    nt, lk = (int(x) for x in a.cfg.split("x"))
    _lib.lib().dtm_jpeg_set_huff(nt, lk)
    dev = torch.device("cuda", 0)
    jp = make_jpegs(a.batch, seed=1)
    batch = jpeg.DeviceBatch([jpeg.scan_prep(j) for j in jp])
    lo, hi = torch.cuda.Stream.priority_range()
    side = torch.cuda.Stream(priority=lo) if a.low_priority else torch.cuda.Stream()
    print("stream priority range (least, greatest) = (%d, %d); decode stream priority %d" % (lo, hi, side.priority))
    torch.manual_seed(1234)
    net = nets_factory.build("resnet_v1_50", num_classes=1000).to(dev)
    step = TrainStep(net, optimizer="momentum", lr=0.1, momentum=0.9)
    x = torch.randn(a.batch, 224, 224, 3, device=dev).to(torch.bfloat16)
    y = torch.randint(0, 1000, (a.batch,), device=dev)
    rgb = torch.empty(max(batch.nrgb, 1), dtype=torch.uint8, device=dev)

    def decode():
        with torch.cuda.stream(side):
            batch.launch(dev, side.cuda_stream, rgb)

    # stand-alone decode time
    decode()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(5):
        decode()
    torch.cuda.synchronize()
    alone = (time.perf_counter() - t) / 5 * 1e3
    for _ in range(5):
        step(x, y)
    torch.cuda.synchronize()
    res = {False: [], True: []}
    for blk in range(2 * a.blocks):
        on = bool(blk % 2)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.steps):
            if on:
                decode()
            step(x, y)
        torch.cuda.synchronize()
        res[on].append((time.perf_counter() - t) / a.steps * 1e3)
    off, on = min(res[False]), min(res[True])
    print("ResNet-50 b%d step: %.3f ms without decode, %.3f ms with a %d-image device decode per step on a side stream "
          "(+%.3f ms, %.2f %%); decode alone %.3f ms (%s%s)" % (a.batch, off, on, a.batch, on - off,
                                                             100.0 * (on - off) / off, alone, a.cfg,
                                                             ", low priority" if a.low_priority else ""))
    print("blocks off:", ["%.3f" % v for v in res[False]], "on:", ["%.3f" % v for v in res[True]])


if __name__ == "__main__":
    main()
