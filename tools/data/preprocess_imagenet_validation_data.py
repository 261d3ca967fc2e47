#!/usr/bin/env python3
"""Move the flat ILSVRC2012 validation images into per-synset sub-directories (reference
inception/data/preprocess_imagenet_validation_data.py).
Usage: preprocess_imagenet_validation_data.py <validation dir> <validation synset labels file>"""
import os
import sys


def main(argv=None):
    argv = sys.argv if argv is None else argv
    if len(argv) < 3:
        print("usage: preprocess_imagenet_validation_data.py <validation data dir> <validation labels file>")
        return 2
    data_dir, labels_file = argv[1], argv[2]
    labels = [l.strip() for l in open(labels_file) if l.strip()]
    for lab in set(labels):
        os.makedirs(os.path.join(data_dir, lab), exist_ok=True)
    for i, lab in enumerate(labels):
        base = "ILSVRC2012_val_%.8d.JPEG" % (i + 1)
        src = os.path.join(data_dir, base)
        if not os.path.exists(src):
            print("Failed to find: %s" % src)
            return 1
        os.rename(src, os.path.join(data_dir, lab, base))
    return 0


if __name__ == "__main__":
    sys.exit(main())
