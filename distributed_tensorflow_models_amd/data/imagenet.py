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
    return np.asarray(Image.open(BytesIO(data)).convert("RGB"))


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


def _resize(img, size, method):
    from PIL import Image
    methods = [Image.BILINEAR, Image.NEAREST, Image.BICUBIC, Image.BOX]  # thread_id % 4 (image_processing.py)
    return np.asarray(Image.fromarray(img).resize((size, size), methods[method % 4]))


def distort_color(img, rng, thread_id=0):
    x = img.astype(np.float32) / 255.0
    ops = [lambda v: v + rng.uniform(-32.0 / 255, 32.0 / 255),
           lambda v: _saturation(v, rng.uniform(0.5, 1.5)),
           lambda v: _hue(v, rng.uniform(-0.2, 0.2)),
           lambda v: (v - v.mean((0, 1), keepdims=True)) * rng.uniform(0.5, 1.5) + v.mean((0, 1), keepdims=True)]
    order = [0, 1, 2, 3] if thread_id % 2 == 0 else [0, 2, 1, 3]  # the two orderings of distort_color
    if thread_id % 2 == 0:
        order = [0, 1, 2, 3]
    else:
        order = [0, 1, 3, 2]
    for k in order:
        x = ops[k](x)
    return np.clip(x, 0.0, 1.0)


def _saturation(x, f):
    gray = x.mean(-1, keepdims=True)
    return gray + (x - gray) * f


def _hue(x, delta):
    # rotate in YIQ space (approximation of tf.image.adjust_hue)
    t = delta * 2 * np.pi
    c, s = np.cos(t), np.sin(t)
    yiq = np.array([[0.299, 0.587, 0.114], [0.596, -0.274, -0.322], [0.211, -0.523, 0.312]], np.float32)
    rot = np.array([[1, 0, 0], [0, c, -s], [0, s, c]], np.float32)
    m = np.linalg.inv(yiq) @ rot @ yiq
    return x @ m.T.astype(np.float32)


def distort_image(img, size, bbox, rng, thread_id=0):
    h, w = img.shape[:2]
    y0, x0, ch, cw = sample_distorted_bounding_box(h, w, bbox, rng)
    crop = img[y0:y0 + ch, x0:x0 + cw]
    out = _resize(crop, size, thread_id)
    if rng.randint(2):
        out = out[:, ::-1]
    return distort_color(out, rng, thread_id)


def eval_image(img, size, central_fraction=0.875):
    h, w = img.shape[:2]
    ch, cw = int(h * central_fraction), int(w * central_fraction)
    y0, x0 = (h - ch) // 2, (w - cw) // 2
    return _resize(img[y0:y0 + ch, x0:x0 + cw], size, 0).astype(np.float32) / 255.0


def image_preprocessing(record, train, size, rng, thread_id=0):
    data, label, bbox, _ = parse_example_proto(record)
    img = _decode_jpeg(data)
    x = distort_image(img, size, bbox, rng, thread_id) if train else eval_image(img, size)
    return (x * 2.0 - 1.0).astype(np.float32), label  # [-1, 1]


class BatchInputs:
    """num_readers x num_preprocess_threads pipeline producing (images [B,S,S,3], labels [B])."""

    def __init__(self, dataset, batch_size, train=True, image_size=299, num_preprocess_threads=4, num_readers=4,
                 queue_batches=4, seed=0, device="cpu", shuffle_buffer=1024):
        self.files = dataset.data_files()
        self.B, self.S, self.train, self.device = batch_size, image_size, train, torch.device(device)
        self.records = queue.Queue(maxsize=shuffle_buffer)
        self.examples = queue.Queue(maxsize=batch_size * queue_batches)
        self.stop = threading.Event()
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
                for rec in tf_record_iterator(f):
                    if self.stop.is_set():
                        return
                    self.records.put(rec)
            if not self.train:
                break

    def _prep(self, tid, seed):
        rng = np.random.RandomState(seed)
        while not self.stop.is_set():
            try:
                rec = self.records.get(timeout=0.5)
            except queue.Empty:
                continue
            self.examples.put(image_preprocessing(rec, self.train, self.S, rng, tid))

    def next_batch(self):
        xs, ys = zip(*[self.examples.get() for _ in range(self.B)])
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
