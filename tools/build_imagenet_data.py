#!/usr/bin/env python3
"""Convert an ImageNet-style image folder tree to sharded TFRecords of tf.train.Example
(reference inception/data/build_imagenet_data.py) without TensorFlow.

  <train_directory>/<synset>/<image>.JPEG  ->  <output_directory>/train-00000-of-01024 ...
Example schema: image/height, width, colorspace, channels, class/label (1-based; 0 = background),
class/synset, class/text, object/bbox/{xmin,xmax,ymin,ymax,label}, format, filename, encoded.
PNG and CMYK JPEG inputs are re-encoded as RGB JPEG (ImageCoder); file order is shuffled with
seed 12345; shards are written by ``--num_threads`` threads, each owning a contiguous shard range.
"""
import argparse
import csv
import io
import os
import random
import sys
import threading

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_tensorflow_models_amd.data.tfrecord import TFRecordWriter, encode_example  # noqa: E402


def _process_image(path):
    from PIL import Image
    raw = open(path, "rb").read()
    img = Image.open(io.BytesIO(raw))
    if img.format != "JPEG" or img.mode != "RGB":  # PNG -> JPEG, CMYK -> RGB
        buf = io.BytesIO()
        img.convert("RGB").save(buf, format="JPEG", quality=100)
        raw = buf.getvalue()
        img = Image.open(io.BytesIO(raw))
    return raw, img.size[1], img.size[0]


def _example(path, label, synset, human, bboxes):
    data, h, w = _process_image(path)
    f = {"image/height": h, "image/width": w, "image/colorspace": b"RGB", "image/channels": 3,
         "image/class/label": label, "image/class/synset": synset.encode(), "image/class/text": human.encode(),
         "image/format": b"JPEG", "image/filename": os.path.basename(path).encode(), "image/encoded": data}
    if bboxes:
        f["image/object/bbox/xmin"] = [float(b[0]) for b in bboxes]
        f["image/object/bbox/ymin"] = [float(b[1]) for b in bboxes]
        f["image/object/bbox/xmax"] = [float(b[2]) for b in bboxes]
        f["image/object/bbox/ymax"] = [float(b[3]) for b in bboxes]
        f["image/object/bbox/label"] = [label] * len(bboxes)
    return encode_example(f)


def find_image_files(data_dir, labels_file=None):
    if labels_file and os.path.exists(labels_file):
        synsets = [l.strip() for l in open(labels_file) if l.strip()]
    else:
        synsets = sorted(d for d in os.listdir(data_dir) if os.path.isdir(os.path.join(data_dir, d)))
    files, labels, syns = [], [], []
    for i, s in enumerate(synsets):
        d = os.path.join(data_dir, s)
        if not os.path.isdir(d):
            continue
        for f in sorted(os.listdir(d)):
            files.append(os.path.join(d, f))
            labels.append(i + 1)  # label 0 is the background class
            syns.append(s)
    order = list(range(len(files)))
    random.Random(12345).shuffle(order)
    return [files[i] for i in order], [labels[i] for i in order], [syns[i] for i in order]


def build_synset_lookup(metadata_file):
    out = {}
    if metadata_file and os.path.exists(metadata_file):
        for line in open(metadata_file):
            parts = line.rstrip("\n").split("\t")
            if len(parts) == 2:
                out[parts[0]] = parts[1]
    return out


def build_bbox_lookup(bbox_file):
    out = {}
    if bbox_file and os.path.exists(bbox_file):
        for row in csv.reader(open(bbox_file)):
            if len(row) == 5:
                out.setdefault(row[0], []).append([float(v) for v in row[1:]])
    return out


def process_dataset(name, directory, num_shards, out_dir, num_threads, labels_file, humans, bboxes):
    files, labels, syns = find_image_files(directory, labels_file)
    os.makedirs(out_dir, exist_ok=True)
    num_threads = max(1, min(num_threads, num_shards))
    shards_per_thread = num_shards // num_threads
    assert shards_per_thread * num_threads == num_shards, "num_shards must be a multiple of num_threads"
    bounds = [int(round(len(files) * s / float(num_shards))) for s in range(num_shards + 1)]

    def work(t):
        for s in range(t * shards_per_thread, (t + 1) * shards_per_thread):
            path = os.path.join(out_dir, "%s-%.5d-of-%.5d" % (name, s, num_shards))
            with TFRecordWriter(path) as w:
                for i in range(bounds[s], bounds[s + 1]):
                    w.write(_example(files[i], labels[i], syns[i], humans.get(syns[i], syns[i]),
                                     bboxes.get(os.path.basename(files[i]))))

    th = [threading.Thread(target=work, args=(t,)) for t in range(num_threads)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    return len(files)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--train_directory", default="/tmp/")
    ap.add_argument("--validation_directory", default="/tmp/")
    ap.add_argument("--output_directory", default="/tmp/")
    ap.add_argument("--train_shards", type=int, default=1024)
    ap.add_argument("--validation_shards", type=int, default=128)
    ap.add_argument("--num_threads", type=int, default=8)
    ap.add_argument("--labels_file", default="imagenet_lsvrc_2015_synsets.txt")
    ap.add_argument("--imagenet_metadata_file", default="imagenet_metadata.txt")
    ap.add_argument("--bounding_box_file", default="./imagenet_2012_bounding_boxes.csv")
    a = ap.parse_args(argv)
    humans = build_synset_lookup(a.imagenet_metadata_file)
    bboxes = build_bbox_lookup(a.bounding_box_file)
    n = process_dataset("validation", a.validation_directory, a.validation_shards, a.output_directory,
                        a.num_threads, a.labels_file, humans, bboxes)
    m = process_dataset("train", a.train_directory, a.train_shards, a.output_directory, a.num_threads,
                        a.labels_file, humans, bboxes)
    print("wrote %d validation and %d train examples" % (n, m))


if __name__ == "__main__":
    main()
