"""Extract numeric ``T(...)`` literals from a reference Scala spec into JSON test fixtures.

Usage: python tools/extract_scala_fixture.py SPEC START END OUT.json
Every ``Tensor[Float](T(...))`` literal between lines START and END is parsed in order; the list of nested
arrays is written to OUT.json. Only numeric data is taken from the spec (it is test data, not code).
"""
import json
import re
import sys


def literals(text):
    out = []
    i = 0
    while True:
        j = text.find("T(", i)
        if j < 0:
            return out
        if j > 0 and (text[j - 1].isalnum() or text[j - 1] == "_"):
            i = j + 2
            continue
        depth, k = 0, j + 1
        while k < len(text):
            if text[k] == "(":
                depth += 1
            elif text[k] == ")":
                depth -= 1
                if depth == 0:
                    break
            k += 1
        lit = text[j:k + 1]
        s = re.sub(r"\bT\(", "[", lit).replace(")", "]")
        s = re.sub(r"(?<=[0-9.])f\b", "", s)
        try:
            out.append(json.loads(s))
        except json.JSONDecodeError:
            pass
        i = k + 1


if __name__ == "__main__":
    spec, a, b, dst = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    lines = open(spec).read().split("\n")[a - 1:b]
    data = literals("\n".join(lines))
    json.dump(data, open(dst, "w"))
    print(len(data), [len(json.dumps(d)) for d in data])
