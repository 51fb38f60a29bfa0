"""Hadoop SequenceFile image records (BGRImgToLocalSeqFile / SeqFileFolder parity) and the native C++ batch
assembler (csrc/host_runtime.cpp) against a plain torch reference."""
import random

import torch

from bigdl_amd.dataset import seqfile as SF
from bigdl_amd.dataset.image import ByteRecord, encode_bgr_record


def test_hadoop_vlong_encoding():
    # values from org.apache.hadoop.io.WritableUtils.writeVLong
    assert SF.write_vlong(0) == b"\x00"
    assert SF.write_vlong(127) == b"\x7f"
    assert SF.write_vlong(-112) == b"\x90"
    assert SF.write_vlong(128) == b"\x8f\x80"
    assert SF.write_vlong(255) == b"\x8f\xff"
    assert SF.write_vlong(256) == b"\x8e\x01\x00"
    assert SF.write_vlong(-113) == b"\x87\x70"
    for v in [0, 1, 127, 128, 300, 65536, -1, -112, -113, -70000, 2 ** 40]:
        assert SF.read_vlong(SF.write_vlong(v), 0)[0] == v


def test_seqfile_roundtrip_with_sync_markers(tmp_path):
    random.seed(0)
    imgs = [(torch.randint(0, 256, (5 + i % 3, 7, 3), dtype=torch.uint8), i % 4 + 1) for i in range(60)]

    class L:
        def __init__(self, c, l):
            self.content, self._l = c, l

        def label(self):
            return self._l

    names = list(SF.BGRImgToLocalSeqFile(25, str(tmp_path / "part"), hasName=True).apply(
        (L(c, l), f"img{i}.jpg") for i, (c, l) in enumerate(imgs)))
    assert len(names) == 3
    recs = list(SF.LocalSeqFileToBytes().apply(names))
    assert len(recs) == 60
    for (c, l), r in zip(imgs, recs):
        assert r.label == l and torch.equal(SF.decode_bgr_record(r.data), c)
    keys = [k for k, _ in SF.read_sequence_file(names[0])]
    assert SF.read_name(keys[3]) == "img3.jpg" and SF.read_label(keys[3]) == "4"
    ds = SF.SeqFileFolder.files(str(tmp_path), classNum=2, shuffle=False)
    assert ds.size() == sum(1 for _, l in imgs if l <= 2)


def test_native_batch_assembler_matches_reference():
    torch.manual_seed(0)
    imgs = [torch.randint(0, 256, (40 + i, 50, 3), dtype=torch.uint8) for i in range(9)]
    recs = [ByteRecord(encode_bgr_record(im), i + 1) for i, im in enumerate(imgs)]
    mean, std = (120.0, 110.0, 100.0), (60.0, 50.0, 40.0)
    tf = SF.NativeBGRImgToBatch(32, 24, 4, mean, std, train=True, seed=3)
    batches = list(tf.apply(iter(recs)))
    assert [b.size() for b in batches] == [4, 4, 1]
    tf2 = SF.NativeBGRImgToBatch(32, 24, 4, mean, std, train=True, seed=3)
    params = torch.cat([tf2._params(imgs[i:i + 4]) for i in (0, 4, 8)])
    got = torch.cat([b.getInput() for b in batches])
    for i, im in enumerate(imgs):
        y, x, f = params[i].tolist()
        c = im[y:y + 24, x:x + 32].float()
        if f:
            c = c.flip(1)
        ref = (c[..., [2, 1, 0]].permute(2, 0, 1) - torch.tensor(mean).view(3, 1, 1)) / torch.tensor(std).view(3, 1, 1)
        assert torch.allclose(got[i], ref, atol=1e-5)
    assert torch.cat([b.getTarget() for b in batches]).tolist() == [float(i + 1) for i in range(9)]
