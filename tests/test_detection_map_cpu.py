"""Object-detection MAP (reference T/optim/ValidationSpec.scala:231-355 values, pinned)."""
import torch

from bigdl_amd import optim as O
from bigdl_amd.utils.table import Table


def _t(**kw):
    t = Table()
    for k, v in kw.items():
        t[k] = torch.tensor(v, dtype=torch.float32)
    return t


def _T(*items):
    t = Table()
    for i, v in enumerate(items, 1):
        t[i] = v
    return t


GT_BOXES = [[100, 100, 200, 200], [300, 100, 400, 200], [100, 300, 200, 400], [300, 300, 400, 400],
            [210, 210, 230, 290], [1100, 1100, 1200, 1200], [1300, 1100, 1400, 1200], [1100, 1300, 1200, 1400],
            [1300, 1300, 1400, 1400], [1210, 1210, 1230, 1290]]
DET_BOXES = [[110, 90, 210, 190], [310, 110, 410, 210], [320, 290, 420, 390], [210, 310, 290, 410],
             [1110, 1090, 1210, 1190], [1310, 1110, 1410, 1210], [1320, 1290, 1420, 1390], [1210, 1310, 1290, 1410]]


def test_map_voc2010_tensor_and_table_outputs():
    target = _T(_t(is_crowd=[0] * 10, classes=[0, 0, 0, 0, 0, 1, 1, 1, 1, 1], bboxes=GT_BOXES))
    row = [8.0]
    for lab, sc, b in zip([0, 0, 0, 0, 1, 1, 1, 1], [1, 2, 4, 3, 1, 3, 4, 2], DET_BOXES):
        row += [lab, sc] + b
    out = torch.tensor([row])
    r = O.MeanAveragePrecisionObjectDetection(3)(out, target)
    assert abs(r.result()[0] - 0.35) < 1e-5
    table = _T(_t(classes=[0, 0, 0, 0, 1, 1, 1, 1], bboxes=DET_BOXES, scores=[1, 2, 4, 3, 1, 3, 4, 2]))
    r2 = O.MeanAveragePrecisionObjectDetection(3)(table, target)
    assert abs(r2.result()[0] - 0.35) < 1e-5


def test_map_empty_detections_and_empty_targets():
    target = _T(_t(is_crowd=[0] * 5, classes=[0] * 5, bboxes=GT_BOXES[:5]))
    assert O.MeanAveragePrecisionObjectDetection(3)(_T(Table()), target).result()[0] == 0.0
    target2 = _T(_t(is_crowd=[0] * 5, classes=[0] * 5, bboxes=GT_BOXES[:5]), Table())
    out = _T(_t(classes=[0] * 4, bboxes=DET_BOXES[:4], scores=[1, 2, 9, 7]),
             _t(classes=[0] * 4, bboxes=DET_BOXES[4:], scores=[0, 5, 4, 8]))
    r = O.MeanAveragePrecisionObjectDetection(3)(out, target2)
    assert abs(r.result()[0] - 0.123809524) < 1e-7


def test_map_results_merge_across_batches_and_coco_voc_factories():
    target = _T(_t(is_crowd=[0] * 10, classes=[0, 0, 0, 0, 0, 1, 1, 1, 1, 1], bboxes=GT_BOXES))
    table = _T(_t(classes=[0, 0, 0, 0, 1, 1, 1, 1], bboxes=DET_BOXES, scores=[1, 2, 4, 3, 1, 3, 4, 2]))
    whole = O.MeanAveragePrecisionObjectDetection(3)(table, target).result()[0]
    # the same image split into two "batches" merges to the same AP (gt counts add up)
    t1 = _T(_t(is_crowd=[0] * 5, classes=[0] * 5, bboxes=GT_BOXES[:5]))
    t2 = _T(_t(is_crowd=[0] * 5, classes=[1] * 5, bboxes=GT_BOXES[5:]))
    o1 = _T(_t(classes=[0] * 4, bboxes=DET_BOXES[:4], scores=[1, 2, 4, 3]))
    o2 = _T(_t(classes=[1] * 4, bboxes=DET_BOXES[4:], scores=[1, 3, 4, 2]))
    m = O.MeanAveragePrecisionObjectDetection(3)
    assert abs((m(o1, t1) + m(o2, t2)).result()[0] - whole) < 1e-6
    coco = O.MeanAveragePrecision.cocoBBox(3, skipClass=-1)
    rc = coco(table, target)
    assert len(rc.impl) == 10 and 0.0 <= rc.result()[0] <= whole + 1e-6
    assert "MAP_bbox@IOU(0.500:0.050:0.950)" in rc.format()
    voc07 = O.MeanAveragePrecision.pascalVOC(3, useVoc2007=True, skipClass=-1)(table, target).result()[0]
    assert 0.0 < voc07 <= 1.0
    # a perfect detector scores 1 on every variant
    perfect = _T(_t(classes=[0, 0, 0, 0, 0, 1, 1, 1, 1, 1], bboxes=GT_BOXES, scores=list(range(10, 0, -1))))
    for meth in (O.MeanAveragePrecisionObjectDetection(2), O.MeanAveragePrecision.cocoBBox(2, skipClass=-1),
                 O.MeanAveragePrecision.pascalVOC(2, useVoc2007=True, skipClass=-1)):
        assert abs(meth(perfect, target).result()[0] - 1.0) < 1e-6


def test_map_difficult_ground_truth_is_neither_tp_nor_fp():
    target = _T(_t(is_crowd=[0, 1], classes=[0, 0], bboxes=[[0, 0, 10, 10], [100, 100, 110, 110]]))
    out = _T(_t(classes=[0, 0], bboxes=[[0, 0, 10, 10], [100, 100, 110, 110]], scores=[0.9, 0.95]))
    r = O.MeanAveragePrecisionObjectDetection(1)(out, target)
    assert r.gtCntForClass == [1]
    assert len(r.predictForClass[0]) == 1 and r.predictForClass[0][0][1] is True
    assert abs(r.predictForClass[0][0][0] - 0.9) < 1e-6
    assert abs(r.result()[0] - 1.0) < 1e-6
