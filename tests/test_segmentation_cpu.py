"""COCO mask utilities and dataset (reference T/dataset/segmentation/SegmentationDatasetSpec.scala fixtures,
T/resources/coco/cocomini.json)."""
import json
import os

import numpy as np
import pytest
import torch

from bigdl_amd.dataset.segmentation import (COCODataset, MaskUtils, PolyMasks, RLEMasks, binary_to_rle,
                                            rle_to_binary)

FIX = os.path.join(os.path.dirname(__file__), "fixtures")
D = json.load(open(os.path.join(FIX, "coco_maskutils.json")))


def test_string_codec():
    r = MaskUtils.string2RLE(D["compressed1"], 100, 200)
    assert r.counts == D["arr1"] and (r.height, r.width) == (100, 200)
    assert MaskUtils.string2RLE(D["compressed2"], 100, 200).counts == D["arr2"]
    assert MaskUtils.RLE2String(RLEMasks(D["arr2"], 100, 200)) == D["compressed2"]
    assert MaskUtils.RLE2String(RLEMasks(D["arr1"], 100, 200)) == D["compressed1"]


def test_poly_to_rle():
    rle = MaskUtils.poly2RLE(PolyMasks([D["poly1"]], 480, 640), 480, 640)
    tgt = MaskUtils.string2RLE(D["poly1_target"], 480, 640)
    assert len(rle[0].counts) == len(tgt.counts)
    assert all(abs(a - b) <= 1 for a, b in zip(rle[0].counts, tgt.counts))
    rle2 = MaskUtils.poly2RLE(PolyMasks([D["poly2"]], 480, 640), 480, 640)
    assert MaskUtils.RLE2String(rle2[0]) == D["poly2_target"]


def test_merge():
    r1 = MaskUtils.poly2RLE(PolyMasks([D["poly1"]], 480, 640), 480, 640)[0]
    r2 = MaskUtils.poly2RLE(PolyMasks([D["poly2"]], 480, 640), 480, 640)[0]
    merged = MaskUtils.mergeRLEs([r1, r2], False)
    tgt = MaskUtils.string2RLE(D["merge_target"], 480, 640)
    assert len(merged.counts) == len(tgt.counts)
    assert all(abs(a - b) <= 1 for a, b in zip(merged.counts, tgt.counts))


def test_bbox_area_iou():
    r1, r2 = RLEMasks(D["rle1"], 480, 640), RLEMasks(D["rle2"], 480, 640)
    assert r1.bbox == (142.0, 245.0, 486.0 + 141, 111.0 + 244)
    assert r2.bbox == (1.0, 155.0, 639.0, 325.0 + 154)
    assert MaskUtils.bboxIOU(r1.bbox, r2.bbox, False) == np.float32(0.25976165)
    assert MaskUtils.rleArea(r1) == 5976 and MaskUtils.rleArea(r2) == 77429
    assert MaskUtils.rleIOU(r1, r2, True) == np.float32(0.58199465)
    assert abs(MaskUtils.rleIOU(r1, r2, False) - 0.04351471) < 1e-7
    assert abs(MaskUtils.rleIOU(r2, r1, False) - 0.04351471) < 1e-7
    assert MaskUtils.rleIOU(r2, r1, True) == np.float32(0.04491857)


def test_binary_roundtrip():
    rng = np.random.default_rng(0)
    m = (rng.random((37, 23)) > 0.6).astype(np.float32)
    r = binary_to_rle(torch.from_numpy(m))
    assert np.array_equal(rle_to_binary(r), m.astype(np.uint8))
    assert r.area == int(m.sum())
    m[0, 0] = 1
    assert binary_to_rle(m).counts[0] == 0


def test_coco_dataset():
    ds = COCODataset.load(os.path.join(FIX, "cocomini.json"), FIX)
    assert len(ds.images) == 5 and len(ds.annotations) == 6
    img = ds.images[0]
    boxes, cls, masks, crowd = ds.to_targets(img)
    assert boxes.shape[0] == len(img.annotations) == len(masks)
    for a, m in zip(img.annotations, masks):
        assert (m.height, m.width) == (img.height, img.width)
        assert ds.categoryId2Idx(a.categoryId) >= 1
    assert ds.getCategoryByIdx(1) == ds.categories[0]
