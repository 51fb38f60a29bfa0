"""TensorBoard summaries (reference T/visualization/SummarySpec, TrainSummarySpec)."""
import torch

from bigdl_amd import nn
from bigdl_amd import optim as O
from bigdl_amd.dataset.core import DataSet, Sample
from bigdl_amd.visualization import FileReader, TrainSummary, ValidationSummary, crc32c
from bigdl_amd.visualization.tensorboard import read_records
from bigdl_amd.utils import pbwire as pb


def test_crc32c_known_vector():
    assert crc32c(b"123456789") == 0xE3069283


def test_scalar_and_histogram_roundtrip(tmp_path):
    s = TrainSummary(str(tmp_path), "app")
    for i in range(1, 6):
        s.addScalar("Loss", 1.0 / i, i)
    s.addHistogram("w", torch.randn(1000), 3)
    vals = s.readScalar("Loss")
    assert [v[0] for v in vals] == [1, 2, 3, 4, 5]
    assert abs(vals[-1][1] - 0.2) < 1e-6
    s.close()
    files = FileReader.listFiles(str(tmp_path / "app" / "train"))
    recs = list(read_records(files[0]))
    assert pb.Msg(recs[0]).str(3) == "brain.Event:2"
    histo = [pb.Msg(r).msg(5).msgs(1)[0] for r in recs[1:] if pb.Msg(r).msg(5).msgs(1)[0].str(1) == "w"][0]
    h = histo.msg(5)
    assert h.double(3) == 1000 and sum(h.doubles(7)) == 1000


def test_optimizer_writes_train_and_validation_summaries(tmp_path):
    X = torch.randn(32, 4)
    Y = X.sum(1, keepdim=True)
    data = [Sample(X[i], Y[i]) for i in range(32)]
    model = nn.Sequential().add(nn.Linear(4, 1))
    opt = O.Optimizer(model, DataSet.array(data), nn.MSECriterion(), batchSize=8,
                      optimMethod=O.SGD(0.05), endTrigger=O.Trigger.maxEpoch(2))
    ts = TrainSummary(str(tmp_path), "job")
    ts.setSummaryTrigger("LearningRate", O.Trigger.severalIteration(1))
    ts.setSummaryTrigger("Parameters", O.Trigger.severalIteration(4))
    vs = ValidationSummary(str(tmp_path), "job")
    opt.setTrainSummary(ts).setValidationSummary(vs)
    opt.setValidation(O.Trigger.everyEpoch(), DataSet.array(data, shuffle=False), [O.Loss(nn.MSECriterion())], 8)
    opt.optimize()
    loss = ts.readScalar("Loss")
    assert len(loss) == 8 and loss[-1][1] < loss[0][1]
    assert len(ts.readScalar("LearningRate")) == 8
    assert len(vs.readScalar("Loss")) >= 1
