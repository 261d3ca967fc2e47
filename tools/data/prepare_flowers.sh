#!/usr/bin/env bash
# Offline flowers preparation (reference download_and_preprocess_flowers*.sh): expects
# flower_photos.tgz already in RAW_DIR; splits 500 images per class into validation (seed 12345)
# and converts both splits to TFRecords.   bash tools/data/prepare_flowers.sh RAW_DIR OUT_DIR
set -e
RAW=${1:?dir holding flower_photos.tgz}; OUT=${2:?output dir}
here=$(cd "$(dirname "$0")/../.." && pwd)
mkdir -p "$OUT/raw"
tar xzf "$RAW/flower_photos.tgz" -C "$OUT/raw"
python3 - "$OUT" <<'PY'
import os, random, shutil, sys
out = sys.argv[1]
src = os.path.join(out, "raw", "flower_photos")
labels = sorted(d for d in os.listdir(src) if os.path.isdir(os.path.join(src, d)))
rng = random.Random(12345)
for lab in labels:
    files = sorted(os.listdir(os.path.join(src, lab)))
    rng.shuffle(files)
    for split, part in (("validation", files[:500]), ("train", files[500:])):
        d = os.path.join(out, split, lab)
        os.makedirs(d, exist_ok=True)
        for f in part:
            shutil.copy(os.path.join(src, lab, f), d)
open(os.path.join(out, "labels.txt"), "w").write("\n".join(labels) + "\n")
PY
python3 "$here/tools/data/build_image_data.py" --train_directory "$OUT/train" --validation_directory "$OUT/validation" \
  --output_directory "$OUT" --labels_file "$OUT/labels.txt"
