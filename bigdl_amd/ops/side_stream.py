"""Weight-gradient GEMMs on a second HIP stream, concurrent with the data-gradient chain.

Reference: the MKL-DNN backward computes a layer's weight gradient (accGradParameters) strictly after its input
gradient on one thread (S/nn/mkldnn/SpatialConvolution.scala:520-589, S/nn/abstractnn/AbstractModule.scala:282
backward = updateGradInput then accGradParameters). On MI355X every backward kernel of a batch-256 ResNet runs well
below both the MFMA and the HBM roofline (latency-bound tiles, profiles/r2_resnet50_pmc_v2.txt: 13-27 % MFMA busy,
1.5-4 TB/s), and a conv's weight gradient depends on nothing the next layers' backward produces. So the weight
gradient of every GPU convolution is issued on a side stream that first waits for the compute stream (its inputs
— the layer input and the output gradient — are ready there), and the data-gradient chain (dgrad GEMM, BN
backward, next layer) keeps going on the compute stream: the two fill the CUs together.

Ordering rules:
  * the side stream waits on the compute stream before each weight-gradient launch (inputs ready);
  * every tensor the side stream reads that the compute stream allocated is held (``keep``) until the next join, so
    the caching allocator cannot hand its block to a later compute-stream allocation while the GEMM still reads it;
  * the compute stream waits for the side stream (``join``) when the OUTERMOST backward returns (the gradients are
    final for whatever reads them next: the optimizer, a clipping pass, user code), and before a gradient bucket's
    collective is launched (parallel/bucketed.py);
  * inside a HIP-graph capture this is an ordinary fork / join of the capture stream.
On by default (``BIGDL_WGRAD_STREAM=0`` disables): ResNet-50 b256 eager 29.40 -> 27.84 ms/step on one MI355X
(profiles/r3_wgrad_side_stream_ab.txt); extra side streams measured no better.

Queue priority: the compute stream is the critical path (busy ~21.9 of a ~22.1 ms step) and the side stream's
weight gradients only fill around it, so training runs the compute stream at HIGH queue priority
(``priority_compute_stream``, called by TrainStep; ``BIGDL_COMPUTE_PRIO=0`` keeps the default stream): when both
streams have workgroups waiting, the dispatcher takes the data-gradient chain's first. RCCL's streams stay at
normal priority (utils/engine.py). ResNet-50 b256
11,200 -> 11,690 img/s interleaved on one box (profiles/r6_iteration_log.txt). Raising the SIDE stream's priority
instead (``BIGDL_WGRAD_PRIO=-1``, round 3) measured no better: that is the wrong direction.
"""
import os

import torch

_ON = [os.environ.get("BIGDL_WGRAD_STREAM", "1") == "1"]
_N = max(1, int(os.environ.get("BIGDL_WGRAD_STREAMS", "1")))      # round-robin side streams per device
_PRIO = int(os.environ.get("BIGDL_WGRAD_PRIO", "0"))
# BIGDL_WGRAD_CUMASK: restrict the side stream to a subset of the CUs (hipExtStreamCreateWithCUMask) so the weight
# gradients cannot occupy every CU the data-gradient chain needs: "" (default) = all CUs; "stride:K" = every K-th CU;
# "first:N" = CUs 0..N-1; or comma-separated 32-bit hex words
_CUMASK = os.environ.get("BIGDL_WGRAD_CUMASK", "")
_STREAMS = {}
_PENDING = []
_RR = [0]


def _one_queue():
    import bigdl_amd

    return bigdl_amd.graph_one_queue()


def enabled():
    return _ON[0]


def set_enabled(on):
    join()
    _ON[0] = bool(on)


def stream_for(t):
    """The side stream for CUDA tensor ``t``'s device, or None when disabled / not on the GPU."""
    if not _ON[0] or not isinstance(t, torch.Tensor) or not t.is_cuda:
        return None
    if not _one_queue() and torch.cuda.is_current_stream_capturing():
        return None          # forked captures only where graph replays are known to keep the captured order
    dev = t.device.index if t.device.index is not None else torch.cuda.current_device()
    ss = _STREAMS.get(dev)
    if ss is None:
        ss = _STREAMS[dev] = [_new_stream(dev) for _ in range(_N)]
    _RR[0] += 1
    return ss[_RR[0] % len(ss)]


def _cu_mask_words(spec, ncu):
    bits = [False] * ncu
    if spec.startswith("stride:"):
        k = int(spec.split(":")[1])
        for i in range(0, ncu, k):
            bits[i] = True
    elif spec.startswith("first:"):
        for i in range(min(ncu, int(spec.split(":")[1]))):
            bits[i] = True
    else:
        return [int(w, 16) for w in spec.split(",")]
    words = [0] * ((ncu + 31) // 32)
    for i, b in enumerate(bits):
        if b:
            words[i // 32] |= 1 << (i % 32)
    return words


def _new_stream(dev):
    if _CUMASK:
        from . import native

        ncu = torch.cuda.get_device_properties(dev).multi_processor_count
        h = native.get().cu_masked_stream(dev, _cu_mask_words(_CUMASK, ncu))
        return torch.cuda.ExternalStream(h, device=dev)
    return torch.cuda.Stream(device=dev, priority=_PRIO)


_COMPUTE_PRIO = os.environ.get("BIGDL_COMPUTE_PRIO", "-1")
_HP = {}


def _ranks_share_gpus():
    """True when more ranks than visible GPUs run on this node (single-GPU multi-rank rehearsals): raised-priority
    queues of several processes on ONE device measured to serialise against each other (a straggler rank's 600 ms
    spin kernel held the other rank's whole iteration, tests/test_straggler_gpu.py), so the one-process-per-GPU
    priority split is kept to that layout."""
    import torch.distributed as dist

    local = os.environ.get("LOCAL_WORLD_SIZE")          # ranks on THIS node (torch.distributed.run sets it)
    if local:
        ranks = int(local)
    elif dist.is_available() and dist.is_initialized():
        ranks = dist.get_world_size()
    else:
        ranks = int(os.environ.get("WORLD_SIZE", "1"))
    return ranks > max(1, torch.cuda.device_count())


def priority_compute_stream(device):
    """Make a high-priority stream the current stream of ``device`` (once; the old current stream's queued work is
    waited for). No-op when disabled, inside a capture, or when the current stream already has raised priority."""
    try:
        prio = int(_COMPUTE_PRIO)
    except ValueError:
        prio = 0
    dev = torch.device(device)
    if prio >= 0 or dev.type != "cuda" or not torch.cuda.is_available() or torch.cuda.is_current_stream_capturing():
        return None
    if _ranks_share_gpus():
        return None
    cur = torch.cuda.current_stream(dev)
    if cur.priority < 0:
        return cur
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    s = _HP.get(idx)
    if s is None:
        s = _HP[idx] = torch.cuda.Stream(device=idx, priority=prio)
    s.wait_stream(cur)
    torch.cuda.set_stream(s)
    return s


def peer_stream(device):
    """A new stream at the current compute stream's priority, for the straggler drop's control and late-exchange
    streams: work the compute stream waits on should not queue behind it at a lower priority."""
    dev = torch.device(device)
    return torch.cuda.Stream(device=dev, priority=torch.cuda.current_stream(dev).priority)


def begin(s):
    """Make ``s`` wait for the compute stream; returns the compute stream."""
    cur = torch.cuda.current_stream(s.device)
    s.wait_stream(cur)
    if s not in _PENDING:
        _PENDING.append(s)
    return cur


_HELD = []


def keep(s, *ts):
    """Keep compute-stream tensors a side-stream kernel reads alive until the next join. (Not ``record_stream``: that
    makes the caching allocator record and poll one event per tensor and stream at every free — hundreds per step —
    and on ROCm a step with that many outstanding events intermittently ran 4x slower. A join makes the compute stream
    wait for the side stream, so blocks released after it are safe to reuse on the compute stream.)"""
    for t in ts:
        if isinstance(t, torch.Tensor) and t.is_cuda:
            _HELD.append(t)


def pending():
    return bool(_PENDING)


def pending_stream():
    """The one side stream with work not yet joined, or None (none pending, or several)."""
    return _PENDING[0] if len(_PENDING) == 1 else None


def reset():
    """Forget the side streams (after an aborted HIP-graph capture a stream forked into it is not reusable)."""
    _PENDING.clear()
    _STREAMS.clear()
    _HELD.clear()


def join():
    """Compute stream waits for every side stream used since the last join."""
    while _PENDING:
        s = _PENDING.pop()
        torch.cuda.current_stream(s.device).wait_stream(s)
    _HELD.clear()
