"""Schema-driven protobuf codec: text format (prototxt / pbtxt) parser + printer and binary decode/encode into
one canonical representation — a dict ``{field_name: [values]}`` where enum values are their NAME strings and
sub-messages are nested dicts. Schemas are plain tables ``{message: {number: (name, kind, sub)}}``; kinds are
int, uint, int64, bool, float, double, string, bytes, enum (sub = enum table name) and msg (sub = message name).
"""
import re
import struct

from ..utils import pbwire as pb

_VARINT_KINDS = ("int", "uint", "int64", "uint64", "bool", "enum")


class Schema:
    def __init__(self, messages, enums):
        self.messages = messages
        self.enums = enums
        self._by_name = {m: {f[0]: (num,) + tuple(f) for num, f in fields.items()} for m, fields in messages.items()}

    # ------------------------------------------------------------------------------------ binary
    def decode(self, msg_name, buf):
        fields = self.messages[msg_name]
        raw = pb.parse(buf)
        out = {}
        for num, items in raw.items():
            if num not in fields:
                continue
            name, kind, sub = fields[num]
            vals = out.setdefault(name, [])
            for wire, v in items:
                if kind == "msg":
                    vals.append(self.decode(sub, v))
                elif kind in ("string",):
                    vals.append(v.decode("utf-8", "replace"))
                elif kind == "bytes":
                    vals.append(v)
                elif kind == "float":
                    if wire == pb.LEN:
                        vals.extend(struct.unpack(f"<{len(v) // 4}f", v))
                    else:
                        vals.append(struct.unpack("<f", v)[0])
                elif kind == "double":
                    if wire == pb.LEN:
                        vals.extend(struct.unpack(f"<{len(v) // 8}d", v))
                    else:
                        vals.append(struct.unpack("<d", v)[0])
                else:
                    ints = []
                    if wire == pb.LEN:
                        pos = 0
                        while pos < len(v):
                            x, pos = pb.read_varint(v, pos)
                            ints.append(x)
                    elif wire == pb.VARINT:
                        ints.append(v)
                    elif wire == pb.FIXED32:
                        ints.append(struct.unpack("<i", v)[0])
                    else:
                        ints.append(struct.unpack("<q", v)[0])
                    for x in ints:
                        if kind in ("int", "int64") and x >= 1 << 63:
                            x -= 1 << 64
                        if kind == "bool":
                            x = bool(x)
                        elif kind == "enum":
                            x = self.enums[sub].get(x, x)
                        vals.append(x)
        return out

    def encode(self, msg_name, d):
        byname = self._by_name[msg_name]
        out = bytearray()
        for name, vals in d.items():
            if name not in byname:
                continue
            num, _, kind, sub = byname[name]
            vals = vals if isinstance(vals, list) else [vals]
            if kind == "float" and len(vals) > 1:
                out += pb.f_packed_floats(num, vals)
                continue
            for v in vals:
                if kind == "msg":
                    out += pb.f_bytes(num, self.encode(sub, v))
                elif kind in ("string", "bytes"):
                    out += pb.f_bytes(num, v)
                elif kind == "float":
                    out += pb.f_float(num, v)
                elif kind == "double":
                    out += pb.f_double(num, v)
                elif kind == "enum":
                    inv = {n: k for k, n in self.enums[sub].items()}
                    out += pb.f_varint(num, inv[v] if isinstance(v, str) else int(v))
                else:
                    out += pb.f_varint(num, int(v))
        return bytes(out)

    # ------------------------------------------------------------------------------------ text
    def parse_text(self, msg_name, text):
        toks = _tokenize(text)
        d, pos = self._parse_fields(msg_name, toks, 0, top=True)
        return d

    def _parse_fields(self, msg_name, toks, pos, top=False):
        byname = self._by_name.get(msg_name, {})
        out = {}
        while pos < len(toks):
            t = toks[pos]
            if t in ("}", ">"):
                if top:
                    raise ValueError("unbalanced '}' in text proto")
                return out, pos + 1
            name = t
            pos += 1
            if pos < len(toks) and toks[pos] == ":":
                pos += 1
            spec = byname.get(name)
            if pos < len(toks) and toks[pos] in ("{", "<"):
                sub = spec[3] if spec else None
                val, pos = self._parse_fields(sub, toks, pos + 1)
            elif pos < len(toks) and toks[pos] == "[":
                pos += 1
                val = []
                while toks[pos] != "]":
                    if toks[pos] != ",":
                        val.append(_scalar(toks[pos], spec[2] if spec else None))
                    pos += 1
                pos += 1
                out.setdefault(name, []).extend(val)
                continue
            else:
                val = _scalar(toks[pos], spec[2] if spec else None)
                pos += 1
            out.setdefault(name, []).append(val)
            if pos < len(toks) and toks[pos] in (",", ";"):
                pos += 1
        if not top:
            raise ValueError("unterminated message in text proto")
        return out, pos

    def to_text(self, msg_name, d, indent=0):
        byname = self._by_name.get(msg_name, {})
        lines = []
        pad = "  " * indent
        for name, vals in d.items():
            spec = byname.get(name)
            kind = spec[2] if spec else None
            for v in (vals if isinstance(vals, list) else [vals]):
                if isinstance(v, dict):
                    lines.append(f"{pad}{name} {{")
                    lines.append(self.to_text(spec[3] if spec else None, v, indent + 1))
                    lines.append(f"{pad}}}")
                elif kind in ("string", "bytes") or (kind is None and isinstance(v, str) and not v.isupper()):
                    s = v.decode("latin-1") if isinstance(v, bytes) else v
                    lines.append(f'{pad}{name}: "{_escape(s)}"')
                elif isinstance(v, bool):
                    lines.append(f"{pad}{name}: {'true' if v else 'false'}")
                elif isinstance(v, float):
                    lines.append(f"{pad}{name}: {v!r}")
                else:
                    lines.append(f"{pad}{name}: {v}")
        return "\n".join(x for x in lines if x != "")


_TOKEN = re.compile(r'"(?:[^"\\]|\\.)*"|\'(?:[^\'\\]|\\.)*\'|[{}<>\[\]:;,]|[^\s{}<>\[\]:;,"\']+')


def _tokenize(text):
    text = re.sub(r"#[^\n]*", "", text)
    return _TOKEN.findall(text)


def _unescape(s):
    return bytes(s, "latin-1").decode("unicode_escape")


def _escape(s):
    return s.replace("\\", "\\\\").replace('"', '\\"')


def _scalar(tok, kind):
    if tok[0] in "\"'":
        v = _unescape(tok[1:-1])
        return v.encode("latin-1") if kind == "bytes" else v
    if kind in ("float", "double"):
        return float(tok)
    if kind in _VARINT_KINDS and kind not in ("enum", "bool"):
        return int(tok, 0)
    if kind == "bool" or tok in ("true", "false", "True", "False"):
        return tok.lower() == "true"
    if kind == "enum":
        return tok
    try:
        return int(tok, 0)
    except ValueError:
        try:
            return float(tok)
        except ValueError:
            return tok
