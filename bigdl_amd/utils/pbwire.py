"""Minimal protobuf wire-format encoder/decoder (no generated code, no schema compiler).

Used by the TensorBoard event writer/reader (S/visualization/tensorboard/*), and by the Caffe / TensorFlow /
ONNX model importers (S/utils/caffe/CaffeLoader.scala, S/utils/tf/TensorflowLoader.scala,
P/contrib/onnx/onnx_loader.py), whose reference implementations rely on generated protobuf classes.
"""
import struct

VARINT, FIXED64, LEN, FIXED32 = 0, 1, 2, 5


# ---------------------------------------------------------------------------------------------- encoding
def varint(n):
    if n < 0:
        n += 1 << 64
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def key(field, wire):
    return varint((field << 3) | wire)


def f_varint(field, n):
    return key(field, VARINT) + varint(int(n))


def f_double(field, x):
    return key(field, FIXED64) + struct.pack("<d", float(x))


def f_float(field, x):
    return key(field, FIXED32) + struct.pack("<f", float(x))


def f_bytes(field, b):
    if isinstance(b, str):
        b = b.encode("utf-8")
    return key(field, LEN) + varint(len(b)) + b


def f_packed_doubles(field, xs):
    return f_bytes(field, struct.pack(f"<{len(xs)}d", *xs))


def f_packed_floats(field, xs):
    return f_bytes(field, struct.pack(f"<{len(xs)}f", *xs))


def f_packed_varints(field, xs):
    return f_bytes(field, b"".join(varint(int(x)) for x in xs))


# ---------------------------------------------------------------------------------------------- decoding
def read_varint(buf, pos):
    result, shift = 0, 0
    while True:
        b = buf[pos]
        pos += 1
        result |= (b & 0x7F) << shift
        if not b & 0x80:
            return result, pos
        shift += 7


def parse(buf):
    """Decode one message into {field_number: [(wire_type, raw_value), ...]} (raw: int or bytes)."""
    out = {}
    pos, n = 0, len(buf)
    buf = memoryview(buf)
    while pos < n:
        k, pos = read_varint(buf, pos)
        field, wire = k >> 3, k & 7
        if wire == VARINT:
            v, pos = read_varint(buf, pos)
        elif wire == FIXED64:
            v = bytes(buf[pos:pos + 8])
            pos += 8
        elif wire == LEN:
            ln, pos = read_varint(buf, pos)
            v = bytes(buf[pos:pos + ln])
            pos += ln
        elif wire == FIXED32:
            v = bytes(buf[pos:pos + 4])
            pos += 4
        elif wire in (3, 4):   # deprecated groups: skip markers
            continue
        else:
            raise ValueError(f"bad wire type {wire} at {pos}")
        out.setdefault(field, []).append((wire, v))
    return out


class Msg:
    """Convenience accessor over ``parse`` output."""

    def __init__(self, buf):
        self.f = parse(buf) if isinstance(buf, (bytes, bytearray, memoryview)) else buf

    def has(self, field):
        return field in self.f

    def raw(self, field):
        return [v for _, v in self.f.get(field, [])]

    def int(self, field, default=0, signed=True):
        vs = self.raw(field)
        if not vs:
            return default
        v = vs[-1]
        if isinstance(v, bytes):
            v = struct.unpack("<q", v)[0] if len(v) == 8 else struct.unpack("<i", v)[0]
        if signed and v >= 1 << 63:
            v -= 1 << 64
        return v

    def bool(self, field, default=False):
        return bool(self.int(field, int(default)))

    def float(self, field, default=0.0):
        vs = self.raw(field)
        if not vs:
            return default
        v = vs[-1]
        return struct.unpack("<f", v)[0] if len(v) == 4 else struct.unpack("<d", v)[0]

    def double(self, field, default=0.0):
        return self.float(field, default)

    def str(self, field, default=""):
        vs = self.raw(field)
        return vs[-1].decode("utf-8", "replace") if vs else default

    def strs(self, field):
        return [v.decode("utf-8", "replace") for v in self.raw(field)]

    def bytes(self, field, default=b""):
        vs = self.raw(field)
        return vs[-1] if vs else default

    def msg(self, field):
        vs = self.raw(field)
        return Msg(vs[-1]) if vs else None

    def msgs(self, field):
        return [Msg(v) for v in self.raw(field)]

    def ints(self, field, signed=True):
        """Repeated integer field, packed or not."""
        out = []
        for wire, v in self.f.get(field, []):
            if wire == LEN:
                pos = 0
                while pos < len(v):
                    x, pos = read_varint(v, pos)
                    out.append(x - (1 << 64) if signed and x >= 1 << 63 else x)
            elif wire == VARINT:
                out.append(v - (1 << 64) if signed and v >= 1 << 63 else v)
            elif wire == FIXED64:
                out.append(struct.unpack("<q", v)[0])
            else:
                out.append(struct.unpack("<i", v)[0])
        return out

    def floats(self, field):
        """Repeated float field, packed or not."""
        out = []
        for wire, v in self.f.get(field, []):
            if wire == LEN:
                out.extend(struct.unpack(f"<{len(v) // 4}f", v))
            elif wire == FIXED32:
                out.append(struct.unpack("<f", v)[0])
        return out

    def doubles(self, field):
        out = []
        for wire, v in self.f.get(field, []):
            if wire == LEN:
                out.extend(struct.unpack(f"<{len(v) // 8}d", v))
            elif wire == FIXED64:
                out.append(struct.unpack("<d", v)[0])
        return out
