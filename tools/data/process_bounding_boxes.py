#!/usr/bin/env python3
"""ImageNet bounding-box XML annotations -> CSV (reference inception/data/process_bounding_boxes.py,
SURVEY.md C51).  Usage: process_bounding_boxes.py <dir with */*.xml> [synsets file] > boxes.csv

Each output line is ``<image>.JPEG,xmin,ymin,xmax,ymax`` with coordinates scaled to [0, 1] by the
annotated image size (min/max swapped if inverted, clipped to [0, 1]); boxes of synsets outside the
optional synsets file and degenerate boxes are skipped (counts reported on stderr).
"""
import glob
import os
import sys
import xml.etree.ElementTree as ET


def parse_annotation(xml_file):
    try:
        root = ET.parse(xml_file).getroot()
    except ET.ParseError:
        print("Failed to parse: " + xml_file, file=sys.stderr)
        return None, []
    filename = root.findtext("filename")
    size = root.find("size")
    width = float(size.findtext("width"))
    height = float(size.findtext("height"))
    boxes = []
    for obj in root.iter("object"):
        bb = obj.find("bndbox")
        xmin, xmax = float(bb.findtext("xmin")) / width, float(bb.findtext("xmax")) / width
        ymin, ymax = float(bb.findtext("ymin")) / height, float(bb.findtext("ymax")) / height

        def clip(v):
            return min(max(v, 0.0), 1.0)
        boxes.append(dict(label=obj.findtext("name"), xmin=clip(min(xmin, xmax)), xmax=clip(max(xmin, xmax)),
                          ymin=clip(min(ymin, ymax)), ymax=clip(max(ymin, ymax))))
    return filename, boxes


def main(argv=None):
    argv = sys.argv if argv is None else argv
    if len(argv) not in (2, 3):
        print("usage: process_bounding_boxes.py <dir> [synsets-file]", file=sys.stderr)
        return 2
    xml_files = sorted(glob.glob(os.path.join(argv[1], "*", "*.xml")))
    labels = set(l.strip() for l in open(argv[2])) if len(argv) == 3 else None
    skipped_files = skipped_boxes = written = 0
    for path in xml_files:
        label = os.path.basename(os.path.dirname(path))
        if labels is not None and label not in labels:
            skipped_files += 1
            continue
        filename, boxes = parse_annotation(path)
        if filename is None:
            continue
        image = os.path.splitext(os.path.basename(path))[0]
        for b in boxes:
            if (labels is not None and b["label"] not in labels) or b["xmin"] >= b["xmax"] or b["ymin"] >= b["ymax"]:
                skipped_boxes += 1
                continue
            print("%s.JPEG,%.4f,%.4f,%.4f,%.4f" % (image, b["xmin"], b["ymin"], b["xmax"], b["ymax"]))
            written += 1
    print("Wrote %d boxes from %d XML files (skipped %d files, %d boxes)" % (written, len(xml_files), skipped_files,
                                                                         skipped_boxes), file=sys.stderr)
    return 0


if __name__ == "__main__":
    sys.exit(main())
