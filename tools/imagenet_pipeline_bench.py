#!/usr/bin/env python3
"""Sustained throughput of the ImageNet input pipelines from local TFRecord shards:
the GPU pipeline (data/imagenet_gpu.py: threaded JPEG decode + HIP crop/resize/flip/colour kernels)
vs the host pipeline (data/imagenet.py: numpy/PIL preprocessing threads).  Shards of synthetic JPEGs
with ImageNet-like sizes (smooth random content, ~60-120 KB each) are written first.
Usage: python tools/imagenet_pipeline_bench.py [--images 2048] [--batch 128] [--decoders 16]"""
import argparse
import io
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def write_shards(d, n, shards=4, seed=0):
    from PIL import Image

    from distributed_tensorflow_models_amd.data.tfrecord import TFRecordWriter, encode_example
    rng = np.random.RandomState(seed)
    per = (n + shards - 1) // shards
    total = 0
    for s in range(shards):
        with TFRecordWriter(os.path.join(d, "train-%05d-of-%05d" % (s, shards))) as w:
            for i in range(per):
                h, wd = rng.randint(300, 500), rng.randint(300, 500)
                lo = rng.rand(h // 16 + 1, wd // 16 + 1, 3)
                img = np.kron(lo, np.ones((16, 16, 1)))[:h, :wd] * 200 + rng.rand(h, wd, 3) * 55
                b = io.BytesIO()
                Image.fromarray(img.astype(np.uint8)).save(b, format="JPEG", quality=90)
                total += len(b.getvalue())
                w.write(encode_example({"image/encoded": b.getvalue(), "image/class/label": int(rng.randint(1, 1001)),
                                        "image/object/bbox/xmin": [0.1], "image/object/bbox/ymin": [0.1],
                                        "image/object/bbox/xmax": [0.9], "image/object/bbox/ymax": [0.9]}))
    return total / (per * shards)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", type=int, default=2048)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--size", type=int, default=299)
    ap.add_argument("--decoders", type=int, default=16)
    ap.add_argument("--batches", type=int, default=12)
    ap.add_argument("--warm-batches", type=int, default=4)
    ap.add_argument("--host", action="store_true", help="also time the host (numpy) pipeline")
    ap.add_argument("--mode", default="both", choices=("split", "full", "both"),
                    help="JPEG decode: split (host Huffman + HIP IDCT/colour), full (host PIL), both (alternating)")
    args = ap.parse_args()
    import torch

    from distributed_tensorflow_models_amd.data import imagenet, imagenet_gpu
    d = tempfile.mkdtemp(prefix="imnet_")
    avg = write_shards(d, args.images)
    print("wrote %d synthetic JPEGs to %s (avg %.0f KB)" % (args.images, d, avg / 1024), flush=True)
    ds = imagenet.ImagenetData("train", d)
    modes = {"split": [True], "full": [False], "both": [False, True, False, True]}[args.mode]
    for split in modes:
        bi = imagenet_gpu.distorted_inputs(ds, args.batch, num_preprocess_threads=4, image_size=args.size,
                                           num_readers=4, num_decoders=args.decoders, split_decode=split)
        for _ in range(args.warm_batches):  # warm-up (decoder start-up: spawned processes import the package)
            x, _ = bi.next_batch()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(args.batches):
            x, y = bi.next_batch()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        bi.close()
        print("gpu pipeline (%s decode): %.0f img/s sustained (batch %d, %d decoder %s, %dx%d bf16 out)" % (
            "split host-Huffman + HIP IDCT/colour" if split else "full host PIL", args.batches * args.batch / dt,
            args.batch, args.decoders, "threads" if os.environ.get("DTM_DECODE_PROCESSES") == "0" else "processes",
            args.size, args.size), flush=True)
    # device-side cost alone: the two kernels on a resident batch
    from distributed_tensorflow_models_amd.data.imagenet_gpu import gpu_preprocess
    rng = np.random.RandomState(0)
    imgs = [(rng.rand(rng.randint(300, 500), rng.randint(300, 500), 3) * 255).astype(np.uint8)
            for _ in range(args.batch)]
    params = [imagenet.sample_params(im.shape[0], im.shape[1], None, rng, i, True) for i, im in enumerate(imgs)]
    gpu_preprocess(imgs, params, args.size, torch.device("cuda"))
    torch.cuda.synchronize()
    buf, tab = imagenet_gpu.pack_batch(imgs, params)
    bt, tt = torch.from_numpy(buf).pin_memory(), torch.from_numpy(tab.view(np.uint8)).pin_memory()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(10):
        imagenet_gpu._launch(bt, tt, args.batch, args.size, torch.device("cuda"), torch.bfloat16)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / 10
    print("device part (H2D + kernels): %.2f ms / batch of %d = %.0f img/s" % (ms, args.batch, args.batch / ms * 1e3),
          flush=True)
    if args.host:
        hb = imagenet.distorted_inputs(ds, args.batch, num_preprocess_threads=args.decoders, image_size=args.size)
        hb.next_batch()
        t = time.perf_counter()
        for _ in range(3):
            hb.next_batch()
        dt = time.perf_counter() - t
        hb.close()
        print("host pipeline: %.0f img/s (numpy/PIL preprocessing, %d threads)" % (3 * args.batch / dt,
                                                                                   args.decoders), flush=True)


if __name__ == "__main__":
    main()
