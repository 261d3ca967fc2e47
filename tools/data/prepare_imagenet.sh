#!/usr/bin/env bash
# Offline ImageNet preparation (replaces the reference's download_and_preprocess_imagenet.sh /
# download_imagenet.sh).  Nothing is downloaded and no credentials are used: place
# ILSVRC2012_img_train.tar, ILSVRC2012_img_val.tar and (optionally) ILSVRC2012_bbox_train_v2.tar.gz
# in $RAW_DIR first.  Label metadata (synsets, metadata, validation labels) is read from $META_DIR.
#   bash tools/data/prepare_imagenet.sh RAW_DIR OUT_DIR META_DIR
set -e
RAW=${1:?raw tarball dir}; OUT=${2:?output dir}; META=${3:?label metadata dir}
here=$(cd "$(dirname "$0")/../.." && pwd)
mkdir -p "$OUT/train" "$OUT/validation" "$OUT/bounding_boxes"
if [ -f "$RAW/ILSVRC2012_bbox_train_v2.tar.gz" ]; then
  tar xzf "$RAW/ILSVRC2012_bbox_train_v2.tar.gz" -C "$OUT/bounding_boxes"
  python3 "$here/tools/data/process_bounding_boxes.py" "$OUT/bounding_boxes" "$META/imagenet_lsvrc_2015_synsets.txt" \
    > "$OUT/imagenet_2012_bounding_boxes.csv"
fi
tar xf "$RAW/ILSVRC2012_img_val.tar" -C "$OUT/validation"
python3 "$here/tools/data/preprocess_imagenet_validation_data.py" "$OUT/validation" \
  "$META/imagenet_2012_validation_synset_labels.txt"
tar xf "$RAW/ILSVRC2012_img_train.tar" -C "$OUT/train"
for t in "$OUT"/train/*.tar; do
  d="${t%.tar}"; mkdir -p "$d"; tar xf "$t" -C "$d"; rm -f "$t"
done
python3 "$here/tools/build_imagenet_data.py" --train_directory "$OUT/train" --validation_directory "$OUT/validation" \
  --output_directory "$OUT" --labels_file "$META/imagenet_lsvrc_2015_synsets.txt" \
  --imagenet_metadata_file "$META/imagenet_metadata.txt" \
  --bounding_box_file "$OUT/imagenet_2012_bounding_boxes.csv"
