"""COCO SequenceFile records (reference COCOSeqFileGenerator.scala / COCODataset.scala COCOSerializeContext,
COCODeserializer; DataSet.SeqFileFolder.filesToRoiImageFrame): the reference's cocomini.json metadata with
synthetic lossless images of the declared sizes, packed and read back."""
import json
import os
import shutil

import numpy as np
import torch
from PIL import Image

from bigdl_amd.dataset.segmentation import (COCO_MAGIC, COCODataset, COCODeserializer, COCOSerializeContext,
                                            PolyMasks, RLEMasks, dump_image_meta, generate_coco_seq_files,
                                            read_coco_seq_files)
from bigdl_amd.dataset.seqfile import _BYTES, SequenceFileWriter, read_sequence_file

FIX = os.path.join(os.path.dirname(__file__), "fixtures", "cocomini.json")


def _images(meta, root):
    rng = np.random.RandomState(0)
    for im in meta["images"]:
        arr = rng.randint(0, 255, (im["height"], im["width"], 3), dtype=np.uint8)
        name = os.path.splitext(im["file_name"])[0] + ".png"
        im["file_name"] = name
        Image.fromarray(arr).save(os.path.join(root, name))


def test_generate_and_read_back(tmp_path):
    meta = json.load(open(FIX))
    _images(meta, str(tmp_path))
    mpath = tmp_path / "meta.json"
    mpath.write_text(json.dumps(meta))
    files = generate_coco_seq_files(str(mpath), str(tmp_path), str(tmp_path / "seq"), blockSize=2)
    assert len(files) == 3
    ds = COCODataset.load(str(mpath), str(tmp_path))
    recs = {r["fileName"]: r for r in read_coco_seq_files(str(tmp_path / "seq"))}
    assert len(recs) == 5
    for im in ds.images:
        r = recs[im.fileName]
        assert r["originalSize"] == (im.height, im.width, 3)
        rgb = np.asarray(Image.open(im.path).convert("RGB"))
        assert torch.equal(r["image"], torch.from_numpy(rgb[..., ::-1].copy()))
        boxes, cls, masks, crowd = ds.to_targets(im)
        assert torch.equal(r["bboxes"], boxes) and torch.equal(r["classes"], cls)
        assert torch.equal(r["isCrowd"], crowd)
        for got, ann in zip(r["masks"], im.annotations):
            if ann.isCrowd:
                assert isinstance(got, RLEMasks) and got.counts == ann.segmentation.counts
            else:
                assert isinstance(got, PolyMasks)
                for a, b in zip(got.poly, ann.segmentation.poly):
                    assert np.allclose(a, b, atol=1e-4)


def test_record_layout_is_big_endian_with_magic():
    ctx = COCOSerializeContext()
    ctx.dump_string("a.jpg")
    ctx.dump_int(7)
    ctx.dump_float(1.5)
    ctx.dump_bool(True)
    b = ctx.toByteArray()
    assert b[:4] == b"\x00\x00\x00\x05" and b[4:9] == b"a.jpg" and b[9:13] == b"\x00\x00\x00\x07"
    assert b[13:17] == b"\x3f\xc0\x00\x00" and b[17:] == b"\x01"
    d = COCODeserializer(b)
    assert d.getString() == "a.jpg" and d.getInt() == 7 and d.getFloat() == 1.5 and d.getBoolean()
    assert COCO_MAGIC == 0x1F3D4E5A


def test_byteswritable_sequence_file_roundtrip(tmp_path):
    p = str(tmp_path / "x.seq")
    with SequenceFileWriter(p, _BYTES, _BYTES) as w:
        for i in range(300):
            w.append(bytes([i % 256]) * (i + 1), b"v" * (2 * i))
    got = list(read_sequence_file(p))
    assert len(got) == 300 and got[5] == (bytes([5]) * 6, b"v" * 10)
