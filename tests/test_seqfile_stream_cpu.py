"""SequenceFile image stream (dataset/seqfile_stream.py): native record index, parallel byte gather, vectorised crop
parameters, rank sharding, and the raw-batch path through the device feed / Optimizer on the CPU engine."""
import os

import pytest
import torch

from bigdl_amd.dataset.image import encode_bgr_record
from bigdl_amd.dataset.seqfile import SequenceFileWriter, read_label, read_sequence_file


def _write(tmp, nfiles=2, per=7, seed=0):
    g = torch.Generator().manual_seed(seed)
    paths, imgs, labels = [], [], []
    for f in range(nfiles):
        p = os.path.join(tmp, f"part_{f}.seq")
        with SequenceFileWriter(p) as w:
            for i in range(per):
                h = int(torch.randint(24, 40, (1,), generator=g))
                wd = int(torch.randint(24, 40, (1,), generator=g))
                im = torch.randint(0, 256, (h, wd, 3), generator=g, dtype=torch.uint8)
                lab = 1 + (f * per + i) % 5
                key = f"img{f}_{i}\n{lab}" if i % 2 else f"{lab}"
                w.append(key, encode_bgr_record(im))
                imgs.append(im)
                labels.append(float(lab))
        paths.append(p)
    return paths, imgs, labels


def test_native_index_matches_python_reader(tmp_path):
    from bigdl_amd.ops import native

    paths, imgs, labels = _write(str(tmp_path), nfiles=1, per=200)   # > SYNC_INTERVAL: sync markers inside
    buf = torch.from_numpy(__import__("numpy").fromfile(paths[0], dtype="uint8"))
    rec, lab = native.get().seqfile_index(buf)
    py = list(read_sequence_file(paths[0]))
    assert rec.shape[0] == len(py) == 200
    for i, (k, v) in enumerate(py):
        assert float(read_label(k)) == float(lab[i])
        o, h, w = rec[i].tolist()
        assert (h, w) == tuple(imgs[i].shape[:2])
        assert torch.equal(buf[o:o + h * w * 3].reshape(h, w, 3), imgs[i])


def test_gather_bytes_and_batches(tmp_path):
    from bigdl_amd.dataset.seqfile_stream import SeqFileImageStream

    paths, imgs, labels = _write(str(tmp_path))
    ds = SeqFileImageStream(paths, 4, crop=(16, 16), threads=3, rank=0, world=1, pin=False)
    assert ds.size() == 14
    seen = 0
    for mb in ds.data(train=False):
        flat, offs, prm = mb.getInput()
        for j in range(offs.shape[0]):
            H, W = int(prm[j, 0]), int(prm[j, 1])
            got = flat[int(offs[j]):int(offs[j]) + H * W * 3].reshape(H, W, 3)
            assert torch.equal(got, imgs[seen])
            assert float(mb.getTarget()[j]) == labels[seen]
            # centre crop of the fixed size for evaluation
            assert (int(prm[j, 4]), int(prm[j, 5])) == (16, 16)
            assert int(prm[j, 2]) == (H - 16) // 2 and int(prm[j, 6]) == 0
            seen += 1
    assert seen == 14


def test_random_resized_crop_params_are_valid(tmp_path):
    from bigdl_amd.dataset.seqfile_stream import SeqFileImageStream

    paths, _, _ = _write(str(tmp_path), per=30)
    ds = SeqFileImageStream(paths, 8, crop=(16, 16), rank=0, world=1, pin=False, seed=3)
    it = ds.data(train=True)
    flips = []
    for _ in range(20):
        prm = next(it).getInput()[2]
        H, W, y0, x0, ch, cw = (prm[:, i] for i in range(6))
        assert bool(((ch > 0) & (cw > 0) & (y0 >= 0) & (x0 >= 0) & (y0 + ch <= H) & (x0 + cw <= W)).all())
        area = ch * cw / (H * W)
        assert bool((area <= 1.0 + 1e-6).all())
        flips.append(prm[:, 6])
    f = torch.cat(flips)
    assert 0.2 < float(f.mean()) < 0.8


def test_rank_sharding_is_disjoint_and_complete(tmp_path):
    from bigdl_amd.dataset.seqfile_stream import SeqFileImageStream

    paths, _, _ = _write(str(tmp_path), per=9)
    got = []
    for r in range(3):
        ds = SeqFileImageStream(paths, 6, crop=(16, 16), rank=r, world=3, pin=False)
        assert ds.batch == 2
        got.append(set(ds.rec[:, 0].tolist()) and {(int(f), int(o)) for f, o in zip(ds.fid, ds.rec[:, 0])})
    assert sum(len(s) for s in got) == 18
    assert len(got[0] | got[1] | got[2]) == 18


def test_raw_batches_train_through_optimizer_on_cpu(tmp_path):
    """The raw batch is finished by ``on_device`` inside the device feed (host transformer math on the CPU
    engine), and a small conv net trains on it through Optimizer.optimize()."""
    from bigdl_amd import nn
    from bigdl_amd.dataset.seqfile_stream import SeqFileImageStream
    from bigdl_amd.optim.optimizer import Optimizer
    from bigdl_amd.optim.sgd import SGD
    from bigdl_amd.optim.trigger import Trigger

    paths, _, _ = _write(str(tmp_path), per=16)
    ds = SeqFileImageStream(paths, 8, crop=(16, 16), rank=0, world=1, pin=False)
    mb = next(ds.data(train=True)).on_device()
    assert tuple(mb.getInput().shape) == (8, 3, 16, 16) and mb.getInput().dtype == torch.float32
    model = (nn.Sequential().add(nn.SpatialConvolution(3, 4, 3, 3, 2, 2, 1, 1)).add(nn.ReLU())
             .add(nn.View(4 * 8 * 8).setNumInputDims(3)).add(nn.Linear(4 * 8 * 8, 5)).add(nn.LogSoftMax()))
    opt = Optimizer(model, ds, nn.ClassNLLCriterion(), batchSize=None, optimMethod=SGD(0.05),
                    endTrigger=Trigger.maxIteration(6))
    opt.optimize()
    assert opt.state["neval"] >= 6
    assert torch.isfinite(torch.tensor(opt.state["Loss"]))


@pytest.mark.parametrize("bad", [b"XYZ", b"SEQ\x05"])
def test_index_rejects_non_seqfiles(bad):
    from bigdl_amd.ops import native

    with pytest.raises(RuntimeError):
        native.get().seqfile_index(torch.frombuffer(bytearray(bad + b"\x00" * 32), dtype=torch.uint8))
