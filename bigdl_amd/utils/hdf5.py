"""Native HDF5 reader / writer for Keras weight files (no h5py in this environment).

Reference: P/keras/converter.py:32-67 (WeightLoader.load_weights_from_hdf5: ``model_weights`` group or root,
``layer_names`` / ``weight_names`` attributes, one dataset per weight) and the Keras 1.2.2 / 2.x ``save_weights`` /
``model.save`` layout.

Scope — the HDF5 structures h5py writes for those files with the default (earliest) file format:
  * superblock versions 0 and 1 (8-byte offsets / lengths);
  * version-1 object headers with continuation blocks; groups as symbol tables (version-1 B-trees of SNOD
    symbol-table nodes over a local heap);
  * dataspace messages v1 / v2, datatype classes fixed-point, floating-point and fixed-length string;
  * data layout messages v1-v3 with compact and contiguous storage, and chunked storage (v1 B-tree chunk index,
    no filters);
  * attribute messages v1-v3 (scalars and 1-D arrays of numbers or fixed-length strings).
Newer-format objects (version-2 "OHDR" headers, link messages, fractal heaps) and compressed chunks raise a clear
error. ``write_h5`` emits the same subset (superblock 0, symbol-table groups, contiguous datasets), used to
produce Keras-layout weight files and as the test fixture generator. Parity with files written by h5py is
unpinned: neither h5py nor an .h5 fixture exists in this environment.
"""
import struct

import numpy as np

SIG = b"\x89HDF\r\n\x1a\n"
UNDEF = 0xFFFFFFFFFFFFFFFF


class HDF5Error(ValueError):
    pass


# ---------------------------------------------------------------------------------------------- reader
class _Obj:
    def __init__(self, f, addr):
        self.f, self.addr = f, addr
        self.msgs = f._messages(addr)

    @property
    def attrs(self):
        out = {}
        for t, data in self.msgs:
            if t == 0x000C:
                k, v = self.f._attribute(data)
                out[k] = v
        return out


class Dataset(_Obj):
    def __init__(self, f, addr):
        super().__init__(f, addr)
        m = dict((t, d) for t, d in self.msgs)
        self.shape = self.f._dataspace(m[0x0001])
        self.dtype, self._conv = self.f._datatype(m[0x0003])
        self._layout = m[0x0008]
        if 0x000B in m:
            raise HDF5Error("filtered (compressed) datasets are not supported")

    def __getitem__(self, key):
        if key not in ((), Ellipsis, slice(None)):
            return self[()][key]
        return self.f._read_data(self._layout, self.shape, self.dtype, self._conv)

    def __array__(self, dtype=None):
        a = self[()]
        return a.astype(dtype) if dtype is not None else a


class Group(_Obj):
    def __init__(self, f, addr):
        super().__init__(f, addr)
        m = dict((t, d) for t, d in self.msgs)
        if 0x0011 not in m:
            if 0x0006 in m or 0x0002 in m:
                raise HDF5Error("new-style (link message) groups are not supported")
            raise HDF5Error("not a group")
        btree, heap = struct.unpack_from("<QQ", m[0x0011])
        self._links = self.f._group_links(btree, heap)

    def keys(self):
        return list(self._links.keys())

    def __contains__(self, name):
        try:
            self[name]
            return True
        except KeyError:
            return False

    def __getitem__(self, path):
        node = self
        for part in [p for p in path.split("/") if p]:
            if not isinstance(node, Group) or part not in node._links:
                raise KeyError(path)
            node = self.f._open(node._links[part])
        return node


class File(Group):
    """Read-only HDF5 file: ``File(path)["group/dataset"][()]``, ``.attrs``."""

    def __init__(self, path):
        with open(path, "rb") as fh:
            self.buf = fh.read()
        pos = self.buf.find(SIG)
        if pos != 0:
            raise HDF5Error(f"{path}: not an HDF5 file")
        ver = self.buf[8]
        if ver not in (0, 1):
            raise HDF5Error(f"superblock version {ver} is not supported")
        so, sl = self.buf[13], self.buf[14]
        if so != 8 or sl != 8:
            raise HDF5Error("only 8-byte offsets / lengths are supported")
        p = 24 + (4 if ver == 1 else 0)           # after versions, sizes, K values, flags (+ indexed-storage K)
        self.base = struct.unpack_from("<Q", self.buf, p)[0]
        p += 32                                    # base, free-space, EOF, driver addresses
        root_hdr = struct.unpack_from("<Q", self.buf, p + 8)[0]
        self._cache = {}
        Group.__init__(self, self, root_hdr)

    def close(self):
        pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False

    # -- low level
    def _u(self, fmt, off):
        return struct.unpack_from(fmt, self.buf, off)

    def _open(self, addr):
        if addr not in self._cache:
            msgs = dict(self._messages(addr))
            self._cache[addr] = Group(self, addr) if 0x0011 in msgs else Dataset(self, addr)
        return self._cache[addr]

    def _messages(self, addr):
        b = self.buf
        if b[addr:addr + 4] == b"OHDR":
            raise HDF5Error("version-2 object headers are not supported")
        ver, _, nmsg, _, hsize = struct.unpack_from("<BBHII", b, addr)
        if ver != 1:
            raise HDF5Error(f"object header version {ver} is not supported")
        blocks = [(addr + 16, hsize)]
        out = []
        while blocks and len(out) < nmsg:
            start, size = blocks.pop(0)
            p, end = start, start + size
            while p + 8 <= end and len(out) < nmsg:
                mtype, msize, _flags = struct.unpack_from("<HHB", b, p)
                data = b[p + 8:p + 8 + msize]
                if mtype == 0x0010:                      # continuation
                    coff, clen = struct.unpack_from("<QQ", data)
                    blocks.append((coff, clen))
                out.append((mtype, data))
                p += 8 + msize
        return out

    def _heap_name(self, heap, off):
        if self.buf[heap:heap + 4] != b"HEAP":
            raise HDF5Error("bad local heap")
        data_addr = self._u("<Q", heap + 24)[0]
        s = data_addr + off
        e = self.buf.index(b"\0", s)
        return self.buf[s:e].decode()

    def _group_links(self, btree, heap):
        links = {}

        def walk(node):
            b = self.buf
            if b[node:node + 4] != b"TREE":
                raise HDF5Error("bad group B-tree node")
            ntype, level, used = struct.unpack_from("<BBH", b, node + 4)
            p = node + 8 + 16                             # signature+type+level+used, left / right siblings
            children = []
            for _ in range(used):
                p += 8                                    # key (heap offset)
                children.append(struct.unpack_from("<Q", b, p)[0])
                p += 8
            for ch in children:
                if level > 0:
                    walk(ch)
                    continue
                if b[ch:ch + 4] != b"SNOD":
                    raise HDF5Error("bad symbol table node")
                nsym = struct.unpack_from("<H", b, ch + 6)[0]
                q = ch + 8
                for _ in range(nsym):
                    name_off, hdr = struct.unpack_from("<QQ", b, q)
                    links[self._heap_name(heap, name_off)] = hdr
                    q += 40
        walk(btree)
        return links

    @staticmethod
    def _dataspace(d):
        ver, ndim = d[0], d[1]
        if ver == 1:
            p = 8
        elif ver == 2:
            if d[3] == 2:          # null dataspace
                return None
            p = 4
        else:
            raise HDF5Error(f"dataspace version {ver}")
        return tuple(struct.unpack_from(f"<{ndim}Q", d, p)) if ndim else ()

    @staticmethod
    def _datatype(d):
        cls, ver = d[0] & 0x0F, d[0] >> 4
        bits = d[1] | (d[2] << 8) | (d[3] << 16)
        size = struct.unpack_from("<I", d, 4)[0]
        order = ">" if bits & 1 else "<"
        if cls == 0:
            signed = bool(bits & 0x08)
            return np.dtype(f"{order}{'i' if signed else 'u'}{size}"), None
        if cls == 1:
            return np.dtype(f"{order}f{size}"), None
        if cls == 3:
            return np.dtype(f"S{size}"), "str"
        raise HDF5Error(f"datatype class {cls} (version {ver}) is not supported")

    def _read_data(self, layout, shape, dtype, conv):
        ver = layout[0]
        n = int(np.prod(shape)) if shape else 1
        nbytes = n * dtype.itemsize
        if ver in (1, 2):
            ndim, cls = layout[1], layout[2]
            p = 8
            if cls == 0:
                p += 4 * ndim
                size = struct.unpack_from("<I", layout, p)[0]
                raw = layout[p + 4:p + 4 + size]
            else:
                addr = struct.unpack_from("<Q", layout, p)[0]
                if cls == 2:
                    return self._chunked(addr, [struct.unpack_from("<I", layout, p + 8 + 4 * i)[0]
                                                for i in range(ndim)], shape, dtype)
                raw = self.buf[addr:addr + nbytes]
        elif ver == 3:
            cls = layout[1]
            if cls == 0:
                size = struct.unpack_from("<H", layout, 2)[0]
                raw = layout[4:4 + size]
            elif cls == 1:
                addr, size = struct.unpack_from("<QQ", layout, 2)
                raw = self.buf[addr:addr + nbytes] if addr != UNDEF else b"\0" * nbytes
            elif cls == 2:
                ndim = layout[2]
                addr = struct.unpack_from("<Q", layout, 3)[0]
                dims = [struct.unpack_from("<I", layout, 11 + 4 * i)[0] for i in range(ndim)]
                return self._chunked(addr, dims, shape, dtype)
            else:
                raise HDF5Error(f"layout class {cls}")
        else:
            raise HDF5Error(f"data layout version {ver} is not supported")
        arr = np.frombuffer(raw[:nbytes], dtype=dtype).reshape(shape)
        return arr.astype(dtype.newbyteorder("=")) if dtype.kind in "iuf" else arr.copy()

    def _chunked(self, btree, cdims, shape, dtype):
        """Chunked storage without filters: v1 B-tree (type 1) of chunks keyed by their element offsets."""
        nd = len(shape)
        out = np.zeros(shape, dtype=dtype)
        cdims = cdims[:nd]
        csize = int(np.prod(cdims)) * dtype.itemsize

        def walk(node):
            b = self.buf
            if b[node:node + 4] != b"TREE" or b[node + 4] != 1:
                raise HDF5Error("bad chunk B-tree node")
            level, used = b[node + 5], struct.unpack_from("<H", b, node + 6)[0]
            p = node + 24
            ksize = 8 + 8 * (nd + 1)
            for _ in range(used):
                _, fmask = struct.unpack_from("<II", b, p)
                offs = struct.unpack_from(f"<{nd}Q", b, p + 8)
                child = struct.unpack_from("<Q", b, p + ksize)[0]
                if level > 0:
                    walk(child)
                else:
                    if fmask:
                        raise HDF5Error("filtered chunks are not supported")
                    chunk = np.frombuffer(b[child:child + csize], dtype=dtype).reshape(cdims)
                    sl = tuple(slice(o, min(o + c, s)) for o, c, s in zip(offs, cdims, shape))
                    out[sl] = chunk[tuple(slice(0, s.stop - s.start) for s in sl)]
                p += ksize + 8
        walk(btree)
        return out.astype(dtype.newbyteorder("=")) if dtype.kind in "iuf" else out

    def _attribute(self, d):
        ver = d[0]
        nlen, tlen, slen = struct.unpack_from("<HHH", d, 2)
        pad = (lambda x: (x + 7) & ~7) if ver == 1 else (lambda x: x)
        p = 8 + (1 if ver == 3 else 0)
        name = d[p:p + nlen].split(b"\0")[0].decode()
        p += pad(nlen)
        dtype, conv = self._datatype(d[p:p + tlen])
        p += pad(tlen)
        shape = self._dataspace(d[p:p + slen])
        p += pad(slen)
        n = int(np.prod(shape)) if shape else 1
        arr = np.frombuffer(d[p:p + n * dtype.itemsize], dtype=dtype)
        if conv == "str":
            vals = [v.split(b"\0")[0] for v in arr.tolist()]
            return name, (vals if shape else vals[0])
        arr = arr.astype(dtype.newbyteorder("="))
        return name, (arr.reshape(shape) if shape else arr[0])


# ---------------------------------------------------------------------------------------------- writer
def _align8(n):
    return (n + 7) & ~7


def _dt_bytes(arr):
    a = np.asarray(arr)
    if a.dtype.kind == "f":
        size = a.dtype.itemsize
        if size == 4:
            props = struct.pack("<HHBBBBI", 0, 32, 23, 8, 0, 23, 127)
        else:
            props = struct.pack("<HHBBBBI", 0, 64, 52, 11, 0, 52, 1023)
        return bytes([0x11, 0x20, 31 if size == 4 else 63, 0]) + struct.pack("<I", size) + props
    if a.dtype.kind in "iu":
        size = a.dtype.itemsize
        return bytes([0x10, 0x08 if a.dtype.kind == "i" else 0, 0, 0]) + struct.pack("<I", size) + \
            struct.pack("<HH", 0, size * 8)
    if a.dtype.kind == "S":
        return bytes([0x13, 0, 0, 0]) + struct.pack("<I", a.dtype.itemsize)
    raise HDF5Error(f"cannot write dtype {a.dtype}")


def _ds_bytes(shape):
    return bytes([1, len(shape), 0, 0]) + b"\0" * 4 + b"".join(struct.pack("<Q", s) for s in shape)


def _attr_value(v):
    if isinstance(v, (list, tuple)) and v and isinstance(v[0], (str, bytes)):
        bs = [x.encode() if isinstance(x, str) else x for x in v]
        return np.array(bs, dtype=f"S{max(1, max(len(b) for b in bs))}"), (len(bs),)
    if isinstance(v, (str, bytes)):
        b = v.encode() if isinstance(v, str) else v
        return np.array([b], dtype=f"S{max(1, len(b))}"), ()
    a = np.asarray(v)
    return a, a.shape


class _Writer:
    def __init__(self):
        self.out = bytearray()

    def alloc(self, n):
        off = len(self.out)
        self.out += b"\0" * _align8(n)
        return off

    def put(self, off, data):
        self.out[off:off + len(data)] = data

    def header(self, msgs):
        body = b""
        for t, data in msgs:
            body += struct.pack("<HHB3x", t, _align8(len(data)), 0) + data + b"\0" * (_align8(len(data)) - len(data))
        off = self.alloc(16 + len(body))
        self.put(off, struct.pack("<BBHII", 1, 0, len(msgs), 1, len(body)) + b"\0" * 4 + body)
        return off

    def attrs(self, attrs):
        msgs = []
        for k, v in attrs.items():
            a, shape = _attr_value(v)
            name = k.encode() + b"\0"
            dt, ds = _dt_bytes(a), _ds_bytes(shape)
            data = struct.pack("<BBHHH", 1, 0, len(name), len(dt), len(ds))
            data += name + b"\0" * (_align8(len(name)) - len(name))
            data += dt + b"\0" * (_align8(len(dt)) - len(dt))
            data += ds + b"\0" * (_align8(len(ds)) - len(ds))
            data += np.ascontiguousarray(a).astype(a.dtype.newbyteorder("<") if a.dtype.kind in "iuf" else a.dtype) \
                .tobytes()
            msgs.append((0x000C, data))
        return msgs

    def dataset(self, arr, attrs):
        a = np.ascontiguousarray(arr)
        if a.dtype.kind in "iuf":
            a = a.astype(a.dtype.newbyteorder("<"))
        raw = a.tobytes()
        daddr = self.alloc(len(raw))
        self.put(daddr, raw)
        layout = struct.pack("<BBQQ", 3, 1, daddr, len(raw))
        msgs = [(0x0001, _ds_bytes(a.shape)), (0x0003, _dt_bytes(a)), (0x0008, layout)] + self.attrs(attrs)
        return self.header(msgs)

    def group(self, tree):
        """tree: {name: ndarray | subtree, "@attrs": {...}} -> object header address; children sorted by name."""
        attrs = tree.get("@attrs", {})
        children = sorted(k for k in tree if k != "@attrs")
        addrs = {}
        for k in children:
            v = tree[k]
            addrs[k] = self.group(v) if isinstance(v, dict) else self.dataset(v, {})
        # local heap with the names (offset 0 = empty string)
        names = b"\0" * 8
        offs = {}
        for k in children:
            offs[k] = len(names)
            nb = k.encode() + b"\0"
            names += nb + b"\0" * (_align8(len(nb)) - len(nb))
        data_seg = self.alloc(len(names))
        self.put(data_seg, names)
        heap = self.alloc(32)
        self.put(heap, b"HEAP" + bytes([0, 0, 0, 0]) + struct.pack("<QQQ", len(names), UNDEF, data_seg))
        # symbol table nodes of at most 8 entries (leaf K = 4) under one B-tree node (internal K = 16 -> 32 children)
        chunks = [children[i:i + 8] for i in range(0, len(children), 8)] or [[]]
        if len(chunks) > 32:
            raise HDF5Error("groups with more than 256 members are not supported by the writer")
        snods = []
        for ch in chunks:
            s = self.alloc(8 + 40 * 8)
            body = b"SNOD" + bytes([1, 0]) + struct.pack("<H", len(ch))
            for k in ch:
                body += struct.pack("<QQI4x16x", offs[k], addrs[k], 0)
            self.put(s, body)
            snods.append((s, ch))
        tree_node = self.alloc(24 + 16 * 33 + 8)
        body = b"TREE" + bytes([0, 0]) + struct.pack("<H", len(snods) if children else 0) + \
            struct.pack("<QQ", UNDEF, UNDEF)
        body += struct.pack("<Q", 0)
        for s, ch in snods if children else []:
            body += struct.pack("<QQ", s, offs[ch[-1]])
        self.put(tree_node, body)
        return self.header([(0x0011, struct.pack("<QQ", tree_node, heap))] + self.attrs(attrs))


def write_h5(path, tree):
    """Write ``tree`` ({name: numpy array | subtree dict, "@attrs": {attr: value}}) as an HDF5 file."""
    w = _Writer()
    sb = w.alloc(96)
    root = w.group(tree)
    eof = len(w.out)
    root_entry = struct.pack("<QQI4x16x", 0, root, 0)
    w.put(sb, SIG + bytes([0, 0, 0, 0, 0, 8, 8, 0]) + struct.pack("<HHI", 4, 16, 0) +
          struct.pack("<QQQQ", 0, UNDEF, eof, UNDEF) + root_entry)
    with open(path, "wb") as f:
        f.write(bytes(w.out))


def _as_str(v):
    return v.decode() if isinstance(v, bytes) else str(v)


def read_keras_weights(path):
    """{layer name: [weight arrays in weight_names order]} from a Keras ``save_weights`` / ``model.save`` file."""
    with File(path) as f:
        g = f["model_weights"] if "model_weights" in f else f
        out = {}
        for name in [_as_str(n) for n in np.atleast_1d(g.attrs["layer_names"])]:
            lg = g[name]
            wn = [_as_str(n) for n in np.atleast_1d(lg.attrs.get("weight_names", []))]
            out[name] = [np.asarray(lg[w][()]) for w in wn]
        return out


def write_keras_weights(path, weights, layer_names=None, keras_version="1.2.2"):
    """Write {layer name: [arrays]} in the Keras ``save_weights`` layout (weights named <layer>_W, _b, ...)."""
    names = list(layer_names or weights.keys())
    tree = {"@attrs": {"layer_names": names, "backend": "tensorflow", "keras_version": keras_version}}
    for n in names:
        ws = weights.get(n, [])
        wn = [f"{n}_param_{i}" for i in range(len(ws))]
        sub = {"@attrs": {"weight_names": wn} if wn else {}}
        for k, a in zip(wn, ws):
            sub[k] = np.asarray(a)
        tree[n] = sub
    write_h5(path, tree)


__all__ = ["File", "Group", "Dataset", "HDF5Error", "write_h5", "read_keras_weights", "write_keras_weights"]
