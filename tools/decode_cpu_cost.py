#!/usr/bin/env python3
"""Host CPU time per ImageNet training image, per decode mode, on ONE core (single process, single thread;
time.process_time, so waiting does not count): the figure that sizes an input pipeline for a node
(trainer.decode_capacity_check; SURVEY.md C17 / reference inception/image_processing.py:476-503, one decode
stream per worker host).

  full   : what a decoder process does per record in the default mode - tf.train.Example parse, baseline JPEG
           decode to RGB (PIL / libjpeg-turbo: Huffman + dequant + IDCT + upsampling + colour conversion) and the
           per-image crop / flip / colour parameter sampling.
  split  : the DTM_SPLIT_DECODE=1 host share - the same parse and parameter sampling, and only the Huffman decode
           to DCT coefficients (csrc/runtime/jpeg.cpp); dequantisation, IDCT, upsampling and colour conversion run as
           HIP kernels (csrc/kernels/jpeg.hip).
  device : the DTM_SPLIT_DECODE=2 host share - the same parse and parameter sampling, and only the JPEG marker parse +
           byte unstuffing (data/jpeg.py scan_item); the Huffman decode runs on the GPU too (jpeg_huff_kernel).
  huffman: the Huffman decode alone (the part of the split host work that is inherently serial).

Synthetic JPEGs with ImageNet-like geometry (300-500 px sides, quality 90, smooth content + noise; ~70 KB -
ImageNet's train JPEGs average ~110 KB at ~400x350), the same generator as tools/imagenet_pipeline_bench.py.
Usage: python tools/decode_cpu_cost.py [--images 512]"""
import argparse
import io
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def make_jpegs(n, seed=0):
    from PIL import Image
    rng = np.random.RandomState(seed)
    out = []
    for _ in range(n):
        h, w = rng.randint(300, 500), rng.randint(300, 500)
        lo = rng.rand(h // 16 + 1, w // 16 + 1, 3)
        img = np.kron(lo, np.ones((16, 16, 1)))[:h, :w] * 200 + rng.rand(h, w, 3) * 55
        b = io.BytesIO()
        Image.fromarray(img.astype(np.uint8)).save(b, format="JPEG", quality=90)
        out.append(b.getvalue())
    return out


def records(jpegs):
    from distributed_tensorflow_models_amd.data.tfrecord import encode_example
    return [encode_example({"image/encoded": j, "image/class/label": 7, "image/object/bbox/xmin": [0.1],
                            "image/object/bbox/ymin": [0.1], "image/object/bbox/xmax": [0.9],
                            "image/object/bbox/ymax": [0.9]}) for j in jpegs]


def per_image_us(fn, items, reps=2):
    fn(items[0])  # warm (library load, tables)
    best = None
    for _ in range(reps):
        t = time.process_time()
        for it in items:
            fn(it)
        dt = (time.process_time() - t) / len(items) * 1e6
        best = dt if best is None else min(best, dt)
    return best


def measure(n=512):
    from PIL import Image

    from distributed_tensorflow_models_amd.data import jpeg
    from distributed_tensorflow_models_amd.data.tfrecord import decode_example
    jp = make_jpegs(n)
    recs = records(jp)
    rng = np.random.RandomState(0)

    def sample_params():  # the per-image distortion draw of the train path (bbox crop, flip, colour order)
        return (rng.uniform(0.05, 1.0), rng.uniform(0.75, 1.33), rng.randint(2), rng.randint(4), rng.rand(4))

    def full(rec):
        ex = decode_example(rec)
        img = Image.open(io.BytesIO(ex["image/encoded"][0]))
        np.asarray(img.convert("RGB"))
        sample_params()

    coefs = np.empty(1 << 22, np.int16)  # (the decoders reuse one coefficient buffer)

    def split(rec):
        ex = decode_example(rec)
        jpeg.huffman_decode(ex["image/encoded"][0], coefs)
        sample_params()

    stream, segs = np.empty(1 << 22, np.uint8), np.empty(1 << 14, np.int32)

    def device(rec):
        ex = decode_example(rec)
        jpeg.scan_item(ex["image/encoded"][0], stream, segs)
        sample_params()

    res = {"avg_kb": sum(len(j) for j in jp) / len(jp) / 1024.0,
           "full_us": per_image_us(full, recs), "split_us": per_image_us(split, recs),
           "device_us": per_image_us(device, recs),
           "huffman_us": per_image_us(lambda j: jpeg.huffman_decode(j, coefs), jp)}
    for m in ("full", "split", "device"):
        res[m + "_img_s_per_cpu"] = 1e6 / res[m + "_us"]
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", type=int, default=512)
    a = ap.parse_args()
    r = measure(a.images)
    print("%d synthetic JPEGs, avg %.0f KB; host CPU time per image on one core:" % (a.images, r["avg_kb"]))
    print("  full  (parse + PIL decode + params): %7.0f us  -> %6.0f img/s per CPU" % (r["full_us"],
                                                                                      r["full_img_s_per_cpu"]))
    print("  split (parse + Huffman + params)   : %7.0f us  -> %6.0f img/s per CPU" % (r["split_us"],
                                                                                      r["split_img_s_per_cpu"]))
    print("  device (parse + unstuff + params)  : %7.0f us  -> %6.0f img/s per CPU" % (r["device_us"],
                                                                                      r["device_img_s_per_cpu"]))
    print("  huffman alone                      : %7.0f us  (%.0f %% of the full decode)" % (
        r["huffman_us"], 100.0 * r["huffman_us"] / r["full_us"]))
    for name, per_gpu in (("ResNet-50 224", 15000), ("Inception-v3 299", 7400)):
        for mode in ("full", "split", "device"):
            print("  %-17s x 8 GPUs = %6.0f img/s needs %4.0f CPUs (%s)" % (
                name, 8 * per_gpu, 8 * per_gpu / r[mode + "_img_s_per_cpu"], mode))


if __name__ == "__main__":
    main()
