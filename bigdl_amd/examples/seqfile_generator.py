"""Pack image datasets into Hadoop SequenceFiles for the training readers.

Reference: S/models/utils/ImageNetSeqFileGenerator.scala (class-folder images, scaled so the short side is
``scaleTo``, stored as BGR bytes keyed by label / name in ``blockSize``-record files) and
S/models/utils/COCOSeqFileGenerator.scala (COCO instances json + images: key = serialised file name, size and
annotations with a magic number, value = the encoded image bytes; BytesWritable records).

    python -m bigdl_amd.examples seqfile --mode imagenet --folder <root with class dirs> --output <dir>
    python -m bigdl_amd.examples seqfile --mode coco --metaPath instances.json --folder <images> --output <dir>

Without inputs a tiny synthetic dataset of the chosen kind is generated, packed and read back.
"""
import argparse
import json
import os
import tempfile

import numpy as np


def _synthetic_imagenet(root, classes=3, per_class=4):
    from PIL import Image

    rng = np.random.RandomState(0)
    for c in range(classes):
        os.makedirs(os.path.join(root, f"n{c:08d}"), exist_ok=True)
        for i in range(per_class):
            Image.fromarray(rng.randint(0, 255, (40 + 4 * i, 48, 3), dtype=np.uint8)).save(
                os.path.join(root, f"n{c:08d}", f"img{i}.png"))


def _synthetic_coco(root):
    from PIL import Image

    rng = np.random.RandomState(1)
    images, anns = [], []
    for i in range(3):
        h, w = 30 + 5 * i, 40
        name = f"img{i}.png"
        Image.fromarray(rng.randint(0, 255, (h, w, 3), dtype=np.uint8)).save(os.path.join(root, name))
        images.append({"id": i + 1, "height": h, "width": w, "file_name": name})
        anns.append({"id": 10 + i, "image_id": i + 1, "category_id": 18, "area": 50.0, "bbox": [2, 3, 10, 8],
                     "iscrowd": 0, "segmentation": [[2, 3, 12, 3, 12, 11, 2, 11]]})
        anns.append({"id": 20 + i, "image_id": i + 1, "category_id": 1, "area": 12.0, "bbox": [5, 5, 4, 3],
                     "iscrowd": 1, "segmentation": {"counts": [h * 5 + 5, 3, h - 3, 3, h * w], "size": [h, w]}})
    meta = os.path.join(root, "instances.json")
    with open(meta, "w") as f:
        json.dump({"info": {}, "licenses": [], "images": images, "annotations": anns,
                   "categories": [{"id": 1, "name": "person"}, {"id": 18, "name": "dog"}]}, f)
    return meta


def run(args):
    from ..dataset.segmentation import generate_coco_seq_files, read_coco_seq_files
    from ..dataset.seqfile import generate_seq_files, read_label, read_sequence_file

    tmp = tempfile.TemporaryDirectory()
    out_dir = args.output or os.path.join(tmp.name, "seq")
    try:
        if args.mode == "imagenet":
            root = args.folder
            if root is None:
                root = os.path.join(tmp.name, "train")
                _synthetic_imagenet(root)
            files = generate_seq_files(root, out_dir, blockSize=args.blockSize, scaleTo=args.scaleTo,
                                       hasName=args.hasName)
            labels = [read_label(k) for f in files for k, _ in read_sequence_file(f)]
            return {"files": len(files), "records": len(labels), "labels": sorted(set(labels))}
        root = args.folder or tmp.name
        meta = args.metaPath or _synthetic_coco(root)
        files = generate_coco_seq_files(meta, root, out_dir, blockSize=args.blockSize)
        recs = list(read_coco_seq_files(out_dir))
        return {"files": len(files), "records": len(recs),
                "annotations": sum(len(r["classes"]) for r in recs),
                "first": {"fileName": recs[0]["fileName"], "size": recs[0]["originalSize"]} if recs else None}
    finally:
        tmp.cleanup()


def build_parser():
    p = argparse.ArgumentParser(prog="seqfile")
    p.add_argument("--mode", choices=["imagenet", "coco"], default="imagenet")
    p.add_argument("--folder", default=None)
    p.add_argument("--metaPath", default=None)
    p.add_argument("--output", default=None)
    p.add_argument("--blockSize", type=int, default=12800)
    p.add_argument("--scaleTo", type=int, default=256)
    p.add_argument("--hasName", action="store_true")
    return p


def main(argv=None):
    print(run(build_parser().parse_args(argv)))
    return 0
