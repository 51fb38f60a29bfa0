"""TensorFlow sessions over the graph's own input pipeline (reference S/utils/tf/Session.scala train / predict /
saveParameters, TensorflowLoader.checkpoints, Module.tensorflowCheckpoints): a GraphDef with a filename queue, a
TFRecordReaderV2, ParseSingleExample and a batching queue feeding a softmax regression is trained queue-fed; the
trained variables are saved to a bin file and a checkpoint session / loadTF(binFile) reproduce the trained model."""
import numpy as np
import torch

from bigdl_amd.interop.tensorflow import SCHEMA, Session, TensorflowLoader
from bigdl_amd.interop.tf_session import fixed_length_records, load_bin, tfrecord_iterator, write_tfrecords
from bigdl_amd.nn.module import Module
from bigdl_amd.nn.tf import encode_example as example_bytes
from bigdl_amd.optim import SGD, Trigger


def _attr(k, **v):
    return {"key": [k], "value": [v]}


def _node(name, op, inputs=(), **attrs):
    return {"name": [name], "op": [op], "input": list(inputs), "attr": [_attr(k, **v) for k, v in attrs.items()]}


def _tensor(t):
    t = torch.as_tensor(t)
    dt = {torch.float32: "DT_FLOAT", torch.int32: "DT_INT32", torch.int64: "DT_INT64"}[t.dtype]
    return {"dtype": [dt], "tensor_shape": [{"dim": [{"size": [s]} for s in t.shape]}],
            "tensor_content": [t.numpy().tobytes()]}


def _const(name, t):
    tp = _tensor(t)
    return _node(name, "Const", dtype={"type": tp["dtype"]}, value={"tensor": [tp]})


def _string_const(name, vals):
    tp = {"dtype": ["DT_STRING"], "tensor_shape": [{"dim": [{"size": [len(vals)]}]}], "string_val": list(vals)}
    return _node(name, "Const", dtype={"type": ["DT_STRING"]}, value={"tensor": [tp]})


def _queue_graph(record_file, w0):
    F = {"type": ["DT_FLOAT"]}
    return [
        _string_const("filenames", [record_file.encode()]),
        _node("input_producer", "FIFOQueueV2", component_types={"list": [{"type": ["DT_STRING"]}]}),
        _node("input_producer/enqueue", "QueueEnqueueManyV2", ["input_producer", "filenames"]),
        _node("reader", "TFRecordReaderV2"),
        _node("read", "ReaderReadV2", ["reader", "input_producer"]),
        _const("default_x", torch.zeros(4)), _const("default_y", torch.zeros(1, dtype=torch.int64)),
        _node("parse", "ParseSingleExample", ["read:1", "default_x", "default_y"], num_sparse={"i": [0]},
              dense_keys={"list": [{"s": [b"x", b"y"]}]}, Tdense={"list": [{"type": ["DT_FLOAT", "DT_INT64"]}]},
              dense_shapes={"list": [{"shape": [{"dim": [{"size": [4]}]}, {"dim": [{"size": [1]}]}]}]}),
        _node("batch_queue", "FIFOQueueV2", component_types={"list": [{"type": ["DT_FLOAT", "DT_INT64"]}]}),
        _node("batch_queue/enqueue", "QueueEnqueueV2", ["batch_queue", "parse:0", "parse:1"]),
        _const("batch/n", torch.tensor(16, dtype=torch.int32)),
        _node("batch", "QueueDequeueManyV2", ["batch_queue", "batch/n"],
              component_types={"list": [{"type": ["DT_FLOAT", "DT_INT64"]}]}),
        _node("W", "VariableV2", dtype=F, shape={"shape": [{"dim": [{"size": [4]}, {"size": [3]}]}]}),
        _const("W/init", w0), _node("W/Assign", "Assign", ["W", "W/init"], T=F),
        _node("W/read", "Identity", ["W"], T=F),
        _node("b", "VariableV2", dtype=F, shape={"shape": [{"dim": [{"size": [3]}]}]}),
        _const("b/init", torch.zeros(3)), _node("b/Assign", "Assign", ["b", "b/init"], T=F),
        _node("b/read", "Identity", ["b"], T=F),
        _node("matmul", "MatMul", ["batch:0", "W/read"], T=F, transpose_a={"b": [False]}, transpose_b={"b": [False]}),
        _node("logits", "BiasAdd", ["matmul", "b/read"], T=F),
        _const("labels/shape", torch.tensor([-1], dtype=torch.int32)),
        _node("labels", "Reshape", ["batch:1", "labels/shape"], T={"type": ["DT_INT64"]}),
        _node("xent", "SparseSoftmaxCrossEntropyWithLogits", ["logits", "labels"], T=F),
        _const("axis", torch.tensor([0], dtype=torch.int32)),
        _node("loss", "Mean", ["xent:0", "axis"], T=F),
        _node("prob", "Softmax", ["logits"], T=F),
    ]


def _write_data(path, n=96, seed=0):
    rng = np.random.RandomState(seed)
    A = rng.randn(4, 3)
    recs = []
    for _ in range(n):
        x = rng.randn(4).astype(np.float32)
        y = int(np.argmax(x @ A))
        recs.append(example_bytes({"x": x.tolist(), "y": [y]}))
    write_tfrecords(path, recs)
    return recs


def test_tfrecord_and_fixed_length_readers(tmp_path):
    p = str(tmp_path / "r.tfrecord")
    write_tfrecords(p, [b"abc", b"", b"hello"])
    assert list(tfrecord_iterator(p)) == [b"abc", b"", b"hello"]
    f = tmp_path / "fixed.bin"
    f.write_bytes(b"HDR" + b"aaaa" + b"bbbb" + b"cccc" + b"FT")
    assert list(fixed_length_records(str(f), 3, 4, 2)) == [b"aaaa", b"bbbb", b"cccc"]


def test_queue_fed_training_checkpoint_roundtrip(tmp_path):
    rec = str(tmp_path / "train.tfrecord")
    _write_data(rec)
    w0 = torch.randn(4, 3, generator=torch.Generator().manual_seed(1)) * 0.1
    g = {"node": _queue_graph(rec, w0), "versions": [{"producer": [21]}]}
    pb = str(tmp_path / "graph.pb")
    with open(pb, "wb") as f:
        f.write(SCHEMA.encode("GraphDef", g))

    sess = Session(pb)
    before = float(sess.predict(["loss"], batchSize=96).mean())
    sess.train(["loss"], optMethod=SGD(learningRate=0.5), endWhen=Trigger.maxEpoch(30), batchSize=16, loss="loss")
    after = float(sess.predict(["loss"], batchSize=96).mean())
    assert after < 0.6 * before, (before, after)
    vars_ = sess.variables()
    assert set(vars_) == {"W", "b"} and vars_["W"].shape == (4, 3)
    assert not torch.allclose(vars_["W"], w0)
    binf = str(tmp_path / "vars.bin")
    sess.saveParameters(binf)
    saved = load_bin(binf)
    assert torch.allclose(saved["W"], vars_["W"]) and torch.allclose(saved["b"], vars_["b"])
    # a checkpoint session starts from the trained variables
    ck = Module.tensorflowCheckpoints(pb, binf)
    assert abs(float(ck.predict(["loss"], batchSize=96).mean()) - after) < 1e-4
    ck2 = TensorflowLoader.checkpoints(pb, binf)
    ck2.predict(["loss"], batchSize=96)
    assert torch.allclose(ck2.variables()["W"], saved["W"])
    # loadTF with the bin file: the inference graph (batch -> prob) carries the trained weights
    m = Module.loadTF(pb, ["batch"], ["prob"], binFile=binf)
    x = torch.randn(5, 4)
    from bigdl_amd.utils.table import Table
    p = m.forward(Table(x, torch.zeros(5, 1, dtype=torch.int64)))
    ref = torch.softmax(x @ saved["W"] + saved["b"], dim=1)
    assert torch.allclose(p, ref, atol=1e-5)
