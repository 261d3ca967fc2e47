"""ImageNet input pipeline (reference inception/image_processing.py, dataset.py, imagenet_data.py;
SURVEY.md §2.8 C47/C48).

* ``Dataset`` / ``ImagenetData``: subset files ``<data_dir>/<subset>-*`` (TFRecord shards written by
  tools/build_imagenet_data.py), 1000 classes (+1 background label 0), 1,281,167 / 50,000 examples.
* ``parse_example_proto``: image/encoded, image/class/label, image/class/text, bbox lists.
* ``distort_image``: sample_distorted_bounding_box (min_object_covered 0.1, aspect [0.75, 1.33],
  area [0.05, 1.0]) -> resize (method = thread_id % 4) -> random flip; ``distort_color`` (brightness
  32/255, saturation [0.5,1.5], hue 0.2, contrast [0.5,1.5], two orderings); ``eval_image``: central
  87.5 % crop + bilinear resize; output scaled to [-1, 1].
* ``BatchInputs``: reader/decoder thread pool (num_readers x num_preprocess_threads) feeding a
  bounded queue of ready batches (replaces RandomShuffleQueue + batch_join).
JPEG decode uses PIL (available in the image); no network access, so real data must be pre-placed.
"""
import glob
import os
import queue
import random
import threading

import numpy as np
import torch

from .tfrecord import decode_example, tf_record_iterator


class Dataset:
    def __init__(self, name, subset, data_dir):
        assert subset in self.available_subsets(), subset
        self.name, self.subset, self.data_dir = name, subset, data_dir

    def available_subsets(self):
        return ["train", "validation"]

    def num_classes(self):
        raise NotImplementedError

    def num_examples_per_epoch(self):
        raise NotImplementedError

    def data_files(self):
        pattern = os.path.join(self.data_dir, "%s-*" % self.subset)
        files = sorted(glob.glob(pattern))
        if not files:
            raise IOError("No files found for dataset %s/%s at %s" % (self.name, self.subset, self.data_dir))
        return files

    def reader(self):
        return tf_record_iterator


class ImagenetData(Dataset):
    def __init__(self, subset, data_dir="/home/ubuntu/imagenet/data/"):
        super().__init__("ImageNet", subset, data_dir)

    def num_classes(self):
        return 1000

    def num_examples_per_epoch(self):
        return 1281167 if self.subset == "train" else 50000


def parse_example_proto(record):
    f = decode_example(record)
    label = int(f.get("image/class/label", [0])[0])
    bbox = None
    if f.get("image/object/bbox/xmin"):
        bbox = np.stack([f["image/object/bbox/ymin"], f["image/object/bbox/xmin"], f["image/object/bbox/ymax"],
                         f["image/object/bbox/xmax"]], 1).astype(np.float32)
    text = f.get("image/class/text", [b""])[0]
    return f["image/encoded"][0], label, bbox, text


def _decode_jpeg(data):
    from io import BytesIO

    from PIL import Image
    im = Image.open(BytesIO(data))
    if im.mode != "RGB":  # (grayscale / CMYK JPEGs; RGB ones skip the extra copy)
        im = im.convert("RGB")
    return np.asarray(im)


def sample_distorted_bounding_box(h, w, bboxes, rng, min_object_covered=0.1, aspect_ratio_range=(0.75, 1.33),
                                  area_range=(0.05, 1.0), max_attempts=100):
    if bboxes is None or len(bboxes) == 0:
        bboxes = np.array([[0.0, 0.0, 1.0, 1.0]], np.float32)
    box = bboxes[rng.randint(len(bboxes))]
    by0, bx0, by1, bx1 = box[0] * h, box[1] * w, box[2] * h, box[3] * w
    barea = max((by1 - by0) * (bx1 - bx0), 1.0)
    for _ in range(max_attempts):
        ar = rng.uniform(*aspect_ratio_range)
        area = rng.uniform(*area_range) * h * w
        ch = int(round(np.sqrt(area / ar)))
        cw = int(round(np.sqrt(area * ar)))
        if ch < 1 or cw < 1 or ch > h or cw > w:
            continue
        y0 = rng.randint(0, h - ch + 1)
        x0 = rng.randint(0, w - cw + 1)
        iy = max(0, min(y0 + ch, by1) - max(y0, by0))
        ix = max(0, min(x0 + cw, bx1) - max(x0, bx0))
        if iy * ix / barea >= min_object_covered:
            return y0, x0, ch, cw
    return 0, 0, h, w


# ---- TF 1.x image semantics on float [0, 1] images (the host oracle of the GPU pipeline) -----------
# resize_images(method=thread_id % 4) without align_corners / half-pixel centres (the TF 1 "legacy"
# sampling: source coordinate = dst * in / out).  Every method is separable, so the resize is
# Wy @ img @ Wx^T with per-axis weight matrices (the GPU kernel evaluates the same taps directly).
RESIZE_METHODS = ("bilinear", "nearest", "bicubic", "area")
_CUBIC_A = -0.75
_CUBIC_TABLE = 1024  # TF's legacy bicubic quantises the fractional offset to 1/1024


def _cubic_weights(delta):
    """TF legacy resize_bicubic taps for offsets -1, 0, 1, 2 (its coefficient table, Keys a = -0.75)."""
    a = _CUBIC_A
    off = int(np.rint(delta * _CUBIC_TABLE))

    def near(x):  # |x| <= 1
        return ((a + 2) * x - (a + 3)) * x * x + 1

    def far(x):  # 1 < |x| < 2
        return ((a * x - 5 * a) * x + 8 * a) * x - 4 * a
    x = off / _CUBIC_TABLE
    y = (_CUBIC_TABLE - off) / _CUBIC_TABLE
    return far(x + 1.0), near(x), near(y), far(y + 1.0)


def resize_weights(n, out, method):
    """[out, n] float64 weight matrix of one axis."""
    W = np.zeros((out, n), np.float64)
    scale = np.float32(n) / np.float32(out)  # float32 coordinates, as TF's resize kernels compute them
    for o in range(out):
        f = float(np.float32(o) * scale)
        scale_f = float(scale)
        if method == "bilinear":
            i0 = int(np.floor(f))
            i1 = min(i0 + 1, n - 1)
            d = f - i0
            W[o, i0] += 1.0 - d
            W[o, i1] += d
        elif method == "nearest":
            W[o, min(int(np.floor(f)), n - 1)] = 1.0
        elif method == "bicubic":
            i = int(np.floor(f))
            for k, wk in zip((-1, 0, 1, 2), _cubic_weights(f - i)):
                W[o, min(max(i + k, 0), n - 1)] += wk
        else:  # area: fractional box [o*scale, (o+1)*scale)
            f1 = float(np.float32(o + 1) * scale)
            i = int(np.floor(f))
            while i < f1:
                lo, hi = max(f, i), min(f1, i + 1)
                if hi > lo:
                    W[o, min(i, n - 1)] += (hi - lo) / scale_f
                i += 1
    return W


def resize(img, size, method="bilinear"):
    """img [h, w, 3] float -> [size, size, 3] float32 (TF 1 legacy resize_images semantics)."""
    h, w = img.shape[:2]
    wy, wx = resize_weights(h, size, method), resize_weights(w, size, method)
    t = np.tensordot(wy, img.astype(np.float64), axes=(1, 0))            # [size, w, 3]
    return np.tensordot(t, wx, axes=(1, 1)).transpose(0, 2, 1).astype(np.float32)  # [size, size, 3]


def rgb_to_hsv(x):
    r, g, b = x[..., 0], x[..., 1], x[..., 2]
    v = np.max(x, -1)
    rng_ = v - np.min(x, -1)
    s = np.where(v > 0, rng_ / np.where(v > 0, v, 1), 0.0)
    safe = np.where(rng_ > 0, rng_, 1)
    h = np.where(r == v, (g - b) / safe, np.where(g == v, (b - r) / safe + 2.0, (r - g) / safe + 4.0)) / 6.0
    h = np.where(rng_ > 0, h, 0.0)
    h = np.where(h < 0, h + 1.0, h)
    return np.stack([h, s, v], -1)


def hsv_to_rgb(x):
    h, s, v = x[..., 0], x[..., 1], x[..., 2]
    c = s * v
    m = v - c
    dh = h * 6.0
    xx = c * (1.0 - np.abs(np.fmod(dh, 2.0) - 1.0))
    k = np.floor(dh).astype(np.int64) % 6
    z = np.zeros_like(c)
    rgb = np.select([k[..., None] == i for i in range(6)],
                    [np.stack(t, -1) for t in ((c, xx, z), (xx, c, z), (z, c, xx), (z, xx, c), (xx, z, c), (c, z, xx))])
    return rgb + m[..., None]


def adjust_saturation(x, f):
    hsv = rgb_to_hsv(x)
    hsv[..., 1] = np.clip(hsv[..., 1] * f, 0.0, 1.0)
    return hsv_to_rgb(hsv)


def adjust_hue(x, delta):
    hsv = rgb_to_hsv(x)
    h = hsv[..., 0] + delta
    hsv[..., 0] = np.where(h < 0, h + 1.0, np.where(h >= 1.0, h - 1.0, h))
    return hsv_to_rgb(hsv)


def adjust_contrast(x, f):
    m = x.mean((0, 1), keepdims=True)
    return (x - m) * f + m


def sample_params(h, w, bbox, rng, thread_id, train):
    """Per-image random parameters of image_preprocessing (shared by the host oracle and the GPU
    pipeline): crop window, resize method (thread_id % 4), flip, colour factors, colour ordering."""
    if not train:
        # tf.image.central_crop(0.875): start = int((h - h * 0.875) / 2), size = h - 2 * start
        y0, x0 = int((h - h * 0.875) / 2), int((w - w * 0.875) / 2)
        return dict(y0=y0, x0=x0, ch=h - 2 * y0, cw=w - 2 * x0, method=0, flip=0, color=0, ordering=0,
                    bright=0.0, sat=1.0, hue=0.0, contrast=1.0)
    y0, x0, ch, cw = sample_distorted_bounding_box(h, w, bbox, rng)
    return dict(y0=y0, x0=x0, ch=ch, cw=cw, method=thread_id % 4, flip=int(rng.randint(2)), color=1,
                ordering=thread_id % 2, bright=float(rng.uniform(-32.0 / 255, 32.0 / 255)),
                sat=float(rng.uniform(0.5, 1.5)), hue=float(rng.uniform(-0.2, 0.2)),
                contrast=float(rng.uniform(0.5, 1.5)))


def preprocess_with_params(img, size, p):
    """uint8 [h, w, 3] -> float32 [size, size, 3] in [-1, 1] (reference inception/image_processing.py:
    decode -> convert_image_dtype -> distort_image / eval_image -> (x - 0.5) * 2)."""
    x = img.astype(np.float32) / 255.0
    x = x[p["y0"]:p["y0"] + p["ch"], p["x0"]:p["x0"] + p["cw"]]
    x = resize(x, size, RESIZE_METHODS[p["method"]]).astype(np.float64)
    if p["flip"]:
        x = x[:, ::-1]
    if p["color"]:
        # distort_color: ordering 0 = brightness, saturation, hue, contrast; 1 = brightness, contrast,
        # saturation, hue (reference image_processing.py:180-193); then clip to [0, 1]
        x = x + p["bright"]
        if p["ordering"] == 0:
            x = adjust_contrast(adjust_hue(adjust_saturation(x, p["sat"]), p["hue"]), p["contrast"])
        else:
            x = adjust_hue(adjust_saturation(adjust_contrast(x, p["contrast"]), p["sat"]), p["hue"])
        x = np.clip(x, 0.0, 1.0)
    return ((x - 0.5) * 2.0).astype(np.float32)


def distort_image(img, size, bbox, rng, thread_id=0):
    h, w = img.shape[:2]
    return preprocess_with_params(img, size, sample_params(h, w, bbox, rng, thread_id, True))


def eval_image(img, size):
    h, w = img.shape[:2]
    return preprocess_with_params(img, size, sample_params(h, w, None, None, 0, False))


def image_preprocessing(record, train, size, rng, thread_id=0):
    data, label, bbox, _ = parse_example_proto(record)
    img = _decode_jpeg(data)
    x = distort_image(img, size, bbox, rng, thread_id) if train else eval_image(img, size)
    return x, label  # [-1, 1]


class _PipelineError:
    """Sentinel a pipeline thread queues when it dies; next_batch re-raises it (no silent hang)."""

    def __init__(self, msg):
        self.msg = msg


def _log_bad_record(e, n):
    import logging
    if n <= 10 or n % 1000 == 0:
        logging.getLogger(__name__).warning("skipping undecodable ImageNet record (%d so far): %r", n, e)


class BatchInputs:
    """num_readers x num_preprocess_threads pipeline producing (images [B,S,S,3], labels [B])."""

    def __init__(self, dataset, batch_size, train=True, image_size=299, num_preprocess_threads=4, num_readers=4,
                 queue_batches=4, seed=0, device="cpu", shuffle_buffer=1024):
        self.files = dataset.data_files()
        self.B, self.S, self.train, self.device = batch_size, image_size, train, torch.device(device)
        self.records = queue.Queue(maxsize=shuffle_buffer)
        self.examples = queue.Queue(maxsize=batch_size * queue_batches)
        self.stop = threading.Event()
        self.bad_records = 0
        self.threads = []
        for r in range(num_readers):
            t = threading.Thread(target=self._read, args=(r, num_readers, seed + r), daemon=True)
            t.start()
            self.threads.append(t)
        for p in range(num_preprocess_threads):
            t = threading.Thread(target=self._prep, args=(p, seed + 100 + p), daemon=True)
            t.start()
            self.threads.append(t)

    def _read(self, rid, n, seed):
        rng = random.Random(seed)
        files = self.files[rid::n] or self.files
        while not self.stop.is_set():
            if self.train:
                rng.shuffle(files)
            for f in files:
                try:
                    for rec in tf_record_iterator(f):
                        if self.stop.is_set():
                            return
                        self.records.put(rec)
                except Exception as e:  # unreadable / corrupt record file: surface it in next_batch
                    self.examples.put(_PipelineError("reading %s: %r" % (f, e)))
                    return
            # train AND eval loop over the files forever, as string_input_producer without num_epochs
            # does (reference image_processing.py:444-452): repeated eval_once calls never starve

    def _prep(self, tid, seed):
        rng = np.random.RandomState(seed)
        while not self.stop.is_set():
            try:
                rec = self.records.get(timeout=0.5)
            except queue.Empty:
                continue
            try:
                ex = image_preprocessing(rec, self.train, self.S, rng, tid)
            except Exception as e:  # one undecodable record is skipped (and counted), not fatal
                self.bad_records += 1
                _log_bad_record(e, self.bad_records)
                continue
            self.examples.put(ex)

    def next_batch(self):
        got = []
        while len(got) < self.B:
            ex = self.examples.get()
            if isinstance(ex, _PipelineError):
                raise RuntimeError("ImageNet input pipeline failed: %s" % ex.msg)
            got.append(ex)
        xs, ys = zip(*got)
        x = torch.from_numpy(np.stack(xs))
        y = torch.tensor(ys, dtype=torch.int64)
        if self.device.type == "cuda":
            x = x.pin_memory().to(self.device, non_blocking=True).to(torch.bfloat16)
            y = y.to(self.device, non_blocking=True)
        return x, y

    def close(self):
        self.stop.set()


def distorted_inputs(dataset, batch_size, num_preprocess_threads=4, image_size=299, **kw):
    return BatchInputs(dataset, batch_size, True, image_size, num_preprocess_threads, **kw)


def inputs(dataset, batch_size, num_preprocess_threads=4, image_size=299, **kw):
    return BatchInputs(dataset, batch_size, False, image_size, num_preprocess_threads, num_readers=1, **kw)
