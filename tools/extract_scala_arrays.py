"""Extract numeric ``val name = Array(...)`` literals from a reference Scala spec into a JSON fixture.

Usage: python tools/extract_scala_arrays.py SPEC START END OUT.json
Only numeric test data is taken (name -> flat list; repeated names get a ``_2``, ``_3`` suffix).
"""
import json
import re
import sys


def extract(text):
    out = {}
    for m in re.finditer(r"val\s+(\w+)\s*(?::[^=]*)?=\s*(?:Tensor\[?\w*\]?\(Storage\()?Array(?:\[\w+\])?\(", text):
        name = m.group(1)
        k, depth = m.end(), 1
        while k < len(text) and depth:
            if text[k] == "(":
                depth += 1
            elif text[k] == ")":
                depth -= 1
            k += 1
        body = text[m.end(): k - 1]
        body = re.sub(r"//[^\n]*", "", body)
        toks = [t.strip().rstrip("fFdDL") for t in body.replace("\n", " ").split(",") if t.strip()]
        try:
            vals = [float(t) for t in toks]
        except ValueError:
            continue
        key, i = name, 2
        while key in out:
            key, i = f"{name}_{i}", i + 1
        out[key] = vals
    return out


if __name__ == "__main__":
    spec, a, b, dst = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    lines = open(spec).read().split("\n")[a - 1: b]
    json.dump(extract("\n".join(lines)), open(dst, "w"))
