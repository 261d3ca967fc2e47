#!/usr/bin/env python3
"""Generic image folder -> sharded TFRecord converter (reference inception/data/build_image_data.py,
SURVEY.md C50), written on the framework's own TFRecord/Example codec (no TensorFlow).

  <dir>/<label>/<image>  ->  <output_directory>/<name>-00000-of-00002 ...
Labels come from ``--labels_file`` (one label per line; index 1.. in file order; 0 is reserved
for background), the file order is shuffled with seed 12345, and every record carries
image/{height,width,colorspace,channels,class/label,class/text,format,filename,encoded}.
"""
import argparse
import os
import random
import sys
import threading

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributed_tensorflow_models_amd.data.tfrecord import TFRecordWriter, encode_example  # noqa: E402
from tools.build_imagenet_data import _process_image  # noqa: E402  (PNG/CMYK -> RGB JPEG re-encode)


def find_image_files(data_dir, labels_file):
    labels_txt = [l.strip() for l in open(labels_file) if l.strip()]
    files, labels, texts = [], [], []
    for idx, text in enumerate(labels_txt, 1):
        d = os.path.join(data_dir, text)
        if not os.path.isdir(d):
            continue
        for f in sorted(os.listdir(d)):
            files.append(os.path.join(d, f))
            labels.append(idx)
            texts.append(text)
    order = list(range(len(files)))
    random.Random(12345).shuffle(order)
    return [files[i] for i in order], [texts[i] for i in order], [labels[i] for i in order]


def convert_to_example(path, label, text):
    data, h, w = _process_image(path)
    return encode_example({"image/height": h, "image/width": w, "image/colorspace": b"RGB", "image/channels": 3,
                           "image/class/label": label, "image/class/text": text.encode(), "image/format": b"JPEG",
                           "image/filename": os.path.basename(path).encode(), "image/encoded": data})


def process_dataset(name, directory, num_shards, labels_file, out_dir, num_threads):
    files, texts, labels = find_image_files(directory, labels_file)
    os.makedirs(out_dir, exist_ok=True)
    num_threads = max(1, min(num_threads, num_shards))
    if num_shards % num_threads:
        raise ValueError("Please make the num_threads commensurate with num_shards")
    per = num_shards // num_threads
    bounds = [int(round(len(files) * s / float(num_shards))) for s in range(num_shards + 1)]

    def work(t):
        for s in range(t * per, (t + 1) * per):
            with TFRecordWriter(os.path.join(out_dir, "%s-%.5d-of-%.5d" % (name, s, num_shards))) as w:
                for i in range(bounds[s], bounds[s + 1]):
                    w.write(convert_to_example(files[i], labels[i], texts[i]))

    ths = [threading.Thread(target=work, args=(t,)) for t in range(num_threads)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    return len(files)


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--train_directory", default="/tmp/")
    ap.add_argument("--validation_directory", default="/tmp/")
    ap.add_argument("--output_directory", default="/tmp/")
    ap.add_argument("--train_shards", type=int, default=2)
    ap.add_argument("--validation_shards", type=int, default=2)
    ap.add_argument("--num_threads", type=int, default=2)
    ap.add_argument("--labels_file", required=True)
    a = ap.parse_args(argv)
    n = process_dataset("validation", a.validation_directory, a.validation_shards, a.labels_file,
                        a.output_directory, a.num_threads)
    m = process_dataset("train", a.train_directory, a.train_shards, a.labels_file, a.output_directory,
                        a.num_threads)
    print("wrote %d validation and %d train examples" % (n, m))


if __name__ == "__main__":
    main()
