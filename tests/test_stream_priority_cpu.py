"""The prioritised stream layout's host-side rules (ops/side_stream.py): the compute-stream priority split is applied
only with one process per GPU, and it is a no-op without a GPU."""
import torch

from bigdl_amd.ops import side_stream


def test_ranks_share_gpus_counts_node_local_ranks(monkeypatch):
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "2")
    assert side_stream._ranks_share_gpus()
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "1")
    assert not side_stream._ranks_share_gpus()
    # a 2-node job with 8 GPUs per node: 16 ranks in the world, 8 on this node -> one process per GPU
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 8)
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    monkeypatch.setenv("WORLD_SIZE", "16")
    assert not side_stream._ranks_share_gpus()
    monkeypatch.delenv("LOCAL_WORLD_SIZE")
    monkeypatch.setenv("WORLD_SIZE", "9")
    assert side_stream._ranks_share_gpus()


def test_priority_compute_stream_is_a_noop_without_a_gpu():
    assert side_stream.priority_compute_stream("cpu") is None
    if not torch.cuda.is_available():
        assert side_stream.priority_compute_stream("cuda") is None
