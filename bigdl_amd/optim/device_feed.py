"""Host -> device batch feed for the training loop.

Reference: DistriOptimizer's iteration overlaps fetching the next batch with the current one's compute
(S/optim/DistriOptimizer.scala:204-233: the data-fetch task of iteration k+1 runs while iteration k's model
update is in flight). MI355X design:

  * a host thread pulls MiniBatches from the dataset iterator (decode / transform / SampleToMiniBatch) and pins
    their tensors (page-locked memory, so the copy engine can DMA them asynchronously) into a small queue;
  * the host -> device copy of batch k+1 is issued on a dedicated copy stream as soon as batch k is handed to the
    training step, and an event marks its completion; taking batch k+1 makes the compute stream wait on that
    event (a device-side dependency: the host never blocks on the copy);
  * ``record_stream`` tells the caching allocator that the device tensors are used on the compute stream, so their
    blocks are not recycled by the copy stream while the step still reads them.
  * a raw batch (``on_device``, dataset/seqfile_stream.py) is finished on the device right after its copy, on the
    copy stream: the host ships uint8 records and the preprocessing kernel overlaps the running step.
On the CPU engine the feed is the host-thread prefetch alone.
"""
import queue
import threading

import torch

from ..utils.table import Table


def _tensors(a):
    if isinstance(a, torch.Tensor):
        yield a
    elif isinstance(a, Table):
        for _, v in a.items():
            yield from _tensors(v)
    elif isinstance(a, (list, tuple)):
        for v in a:
            yield from _tensors(v)


def _map(a, fn):
    if isinstance(a, torch.Tensor):
        return fn(a)
    if isinstance(a, Table):
        out = Table()
        for k, v in a.items():
            out[k] = _map(v, fn)
        return out
    if isinstance(a, (list, tuple)):
        return type(a)(_map(v, fn) for v in a)
    return a


class DeviceFeed:
    """Iterator of device-resident MiniBatches with the next batch's copy in flight (depth = host queue size)."""

    def __init__(self, it, device, depth=2, pin=True):
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        self.pin = pin and self.cuda
        self._q = queue.Queue(max(1, depth))
        self._done = object()
        self._err = None
        self._stop = False
        self._thread = threading.Thread(target=self._worker, args=(it,), daemon=True)
        self._thread.start()
        self.stream = torch.cuda.Stream(self.device) if self.cuda else None
        self._pending = None
        self.h2d_issued = 0

    # ------------------------------------------------------------------ host side
    def _worker(self, it):
        try:
            for mb in it:
                if self._stop:
                    return
                if self.pin:
                    mb = _rebuild(mb, _map(mb.getInput(), _pin), _map(mb.getTarget(), _pin))
                self._q.put(mb)
        except BaseException as e:  # noqa: BLE001 - re-raised in the consumer
            self._err = e
        finally:
            self._q.put(self._done)

    def _take_host(self):
        mb = self._q.get()
        if mb is self._done:
            self._q.put(self._done)          # keep the end marker for further calls
            if self._err is not None:
                raise self._err
            raise StopIteration
        return mb

    # ------------------------------------------------------------------ device side
    def _issue(self):
        mb = self._take_host()
        if not self.cuda:
            fin = getattr(mb, "on_device", None)
            return (fin() if fin is not None else mb), None
        with torch.cuda.stream(self.stream):
            dev = _rebuild(mb, _map(mb.getInput(), lambda t: t.to(self.device, non_blocking=True)),
                           _map(mb.getTarget(), lambda t: t.to(self.device, non_blocking=True)))
            fin = getattr(dev, "on_device", None)
            if fin is not None:      # raw batch (dataset/seqfile_stream.py): finished by a kernel on this stream
                dev = fin()
            ev = torch.cuda.Event()
            ev.record(self.stream)
        self.h2d_issued += 1
        return (dev, mb), ev          # keep the pinned host batch alive until its copy completed

    def __iter__(self):
        return self

    def __next__(self):
        if self._pending is None:
            self._pending = self._issue()
        item, ev = self._pending
        self._pending = None
        if not self.cuda:
            return item
        dev, _host = item
        cur = torch.cuda.current_stream(self.device)
        cur.wait_event(ev)
        for t in list(_tensors(dev.getInput())) + list(_tensors(dev.getTarget())):
            if t.is_sparse:
                t._indices().record_stream(cur)
                t._values().record_stream(cur)
            else:
                t.record_stream(cur)
        try:
            self._pending = self._issue()     # the next batch's copy overlaps this step
        except StopIteration:
            self._pending = None
        return dev

    def close(self):
        self._stop = True
        try:
            while True:
                self._q.get_nowait()
        except queue.Empty:
            pass


def _rebuild(mb, inp, tgt):
    """Same batch type over new tensors (``rebuild`` keeps a raw batch's configuration)."""
    fn = getattr(mb, "rebuild", None)
    return fn(inp, tgt) if fn is not None else type(mb)(inp, tgt)


def _pin(t):
    if isinstance(t, torch.Tensor) and t.device.type == "cpu" and not t.is_sparse and not t.is_pinned():
        return t.pin_memory()
    return t
