"""TensorBoard event files: TFRecord framing with masked CRC32C, Event/Summary protobufs written by hand.

Reference: S/visualization/tensorboard/{FileWriter.scala:31, EventWriter.scala:31 (background queue flushed by a
writer thread), RecordWriter.scala:31 (uint64 length, masked crc of length, payload, masked crc of payload),
FileReader.scala (readScalar)}, S/utils/Crc32.scala:21 + J/netty/Crc32c.java.
"""
import glob
import os
import queue
import socket
import struct
import threading
import time

from ..utils import pbwire as pb

# ---------------------------------------------------------------------------------------------- crc32c
_POLY = 0x82F63B78
_TABLE = []
for _i in range(256):
    _c = _i
    for _ in range(8):
        _c = (_c >> 1) ^ _POLY if _c & 1 else _c >> 1
    _TABLE.append(_c)


def crc32c(data):
    c = 0xFFFFFFFF
    t = _TABLE
    for b in data:
        c = t[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def masked_crc32c(data):
    c = crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


# ---------------------------------------------------------------------------------------------- protos
def scalar_summary(tag, value):
    """Summary{ value: [Value{tag, simple_value}] }"""
    return pb.f_bytes(1, pb.f_bytes(1, tag) + pb.f_float(2, value))


_LIMITS = None


def _limits():
    global _LIMITS
    if _LIMITS is None:
        pos, v = [], 1e-12
        for _ in range(774):
            pos.append(v)
            v *= 1.1
        _LIMITS = [-x for x in reversed(pos)] + [0.0] + pos
    return _LIMITS


def histogram_summary(tag, values):
    """HistogramProto with the reference's 1549 exponential buckets (Summary.scala makeHistogramBuckets)."""
    import bisect

    import torch

    vals = values.detach().double().reshape(-1).cpu()
    lim = _limits()
    lt = torch.tensor(lim, dtype=torch.float64)
    idx = torch.searchsorted(lt, vals, right=False)
    counts = torch.bincount(idx, minlength=len(lim) + 1)
    limits, buckets = [], []
    for i in torch.nonzero(counts).flatten().tolist():
        limits.append(lim[i] if i < len(lim) else float("inf"))
        buckets.append(float(counts[i]))
    del bisect
    h = (pb.f_double(1, float(vals.min())) + pb.f_double(2, float(vals.max())) + pb.f_double(3, vals.numel())
         + pb.f_double(4, float(vals.sum())) + pb.f_double(5, float((vals * vals).sum()))
         + pb.f_packed_doubles(6, limits) + pb.f_packed_doubles(7, buckets))
    return pb.f_bytes(1, pb.f_bytes(1, tag) + pb.f_bytes(5, h))


def event(step, wall_time=None, summary=None, file_version=None):
    b = pb.f_double(1, time.time() if wall_time is None else wall_time) + pb.f_varint(2, step)
    if file_version is not None:
        b += pb.f_bytes(3, file_version)
    if summary is not None:
        b += pb.f_bytes(5, summary)
    return b


# ---------------------------------------------------------------------------------------------- writers
class RecordWriter:
    def __init__(self, path):
        self.f = open(path, "ab")

    def write(self, data):
        ln = struct.pack("<Q", len(data))
        self.f.write(ln + struct.pack("<I", masked_crc32c(ln)) + data + struct.pack("<I", masked_crc32c(data)))

    def flush(self):
        self.f.flush()

    def close(self):
        self.f.close()


class EventWriter(threading.Thread):
    """Background writer draining a queue of serialized events (EventWriter.scala)."""

    def __init__(self, logdir, flush_secs=1.0):
        super().__init__(daemon=True)
        os.makedirs(logdir, exist_ok=True)
        name = f"bigdl.tfevents.{int(time.time())}.{socket.gethostname()}.{os.getpid()}.{id(self) % 10000}"
        self.path = os.path.join(logdir, name)
        self.rec = RecordWriter(self.path)
        self.rec.write(event(0, file_version="brain.Event:2"))
        self.rec.flush()
        self.q = queue.Queue()
        self.flush_secs = flush_secs
        self._closing = threading.Event()
        self.start()

    def add(self, ev):
        self.q.put(ev)

    def run(self):
        while not self._closing.is_set() or not self.q.empty():
            try:
                ev = self.q.get(timeout=self.flush_secs)
                self.rec.write(ev)
                while not self.q.empty():
                    self.rec.write(self.q.get_nowait())
                self.rec.flush()
            except queue.Empty:
                pass

    def close(self):
        self._closing.set()
        self.join()
        self.rec.close()


class FileWriter:
    def __init__(self, logdir, flush_secs=1.0):
        self.logdir = logdir
        self.writer = EventWriter(logdir, flush_secs)

    def addSummary(self, summary, step):
        self.writer.add(event(step, summary=summary))
        return self

    def flush(self):
        # drain synchronously
        while not self.writer.q.empty():
            time.sleep(0.01)
        time.sleep(0.02)
        self.writer.rec.flush()

    def close(self):
        self.writer.close()


# ---------------------------------------------------------------------------------------------- reader
def read_records(path):
    with open(path, "rb") as f:
        data = f.read()
    pos = 0
    while pos + 12 <= len(data):
        (ln,) = struct.unpack_from("<Q", data, pos)
        (lcrc,) = struct.unpack_from("<I", data, pos + 8)
        if lcrc != masked_crc32c(data[pos:pos + 8]):
            raise IOError(f"{path}: corrupt record length at {pos}")
        rec = data[pos + 12:pos + 12 + ln]
        (dcrc,) = struct.unpack_from("<I", data, pos + 12 + ln)
        if dcrc != masked_crc32c(rec):
            raise IOError(f"{path}: corrupt record at {pos}")
        yield rec
        pos += 12 + ln + 4


class FileReader:
    @staticmethod
    def listFiles(folder):
        return sorted(glob.glob(os.path.join(folder, "*tfevents*")))

    @staticmethod
    def readScalar(folder, tag):
        """[(step, value, wall_time)] of every scalar ``tag`` under ``folder``, ordered by step."""
        out = []
        for path in FileReader.listFiles(folder):
            for rec in read_records(path):
                ev = pb.Msg(rec)
                s = ev.msg(5)
                if s is None:
                    continue
                for v in s.msgs(1):
                    if v.str(1) == tag and v.has(2):
                        out.append((ev.int(2), v.float(2), ev.double(1)))
        out.sort(key=lambda r: r[0])
        return out
