"""Check a dumped HIP graph (BIGDL_GRAPH_DOT=dir, hipGraphDebugDotPrint) for missing orderings: for every kernel node
whose name matches --sink (default: the optimizer update kernel), list the kernel nodes that are neither its
ancestors nor its descendants (nodes that may run concurrently with it). In a stream-captured training step every
backward kernel must be an ancestor of the update.
    python tools/graph_dot_check.py gpurun_out/dot/*.dot [--sink sgd4_kernel]"""
import argparse
import collections
import re


def parse(path):
    txt = open(path, errors="replace").read()
    labels = {}
    for m in re.finditer(r'^\s*"?([A-Za-z0-9_]+)"?\s*\[(.*?)\];?\s*$', txt, re.M | re.S):
        nid, attrs = m.group(1), m.group(2)
        lab = re.search(r'label\s*=\s*"(.*?)"(?:,|\s*$)', attrs, re.S) or re.search(r"label\s*=\s*<(.*?)>", attrs, re.S)
        labels[nid] = lab.group(1) if lab else attrs
    edges = [(a, b) for a, b in re.findall(r'"?([A-Za-z0-9_]+)"?\s*->\s*"?([A-Za-z0-9_]+)"?', txt)]
    return labels, edges


def short(label):
    m = re.search(r"(\w+_kernel|\w+Kernel|\w+_kernel<[^>]*>|MEMSET|MEMCPY|EVENT\w*|EMPTY|memset|memcpy)", label)
    return m.group(1) if m else label[:60].replace("\\n", " ")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("files", nargs="+")
    ap.add_argument("--sink", default="sgd4_kernel")
    a = ap.parse_args()
    for f in a.files:
        labels, edges = parse(f)
        succ, pred = collections.defaultdict(set), collections.defaultdict(set)
        for x, y in edges:
            succ[x].add(y)
            pred[y].add(x)
        nodes = set(labels) | set(succ) | set(pred)

        def closure(n, nbr):
            seen, st = set(), [n]
            while st:
                for m in nbr[st.pop()]:
                    if m not in seen:
                        seen.add(m)
                        st.append(m)
            return seen
        roots = [n for n in nodes if not pred[n]]
        sinks = [n for n in nodes if a.sink in labels.get(n, "")]
        print(f"{f}: {len(nodes)} nodes, {len(edges)} edges, {len(roots)} roots, {len(sinks)} '{a.sink}' nodes")
        for s in sinks:
            anc, dec = closure(s, pred), closure(s, succ)
            free = [n for n in nodes if n != s and n not in anc and n not in dec]
            kinds = collections.Counter(short(labels.get(n, n)) for n in free)
            print(f"  {s}: ancestors {len(anc)}, descendants {len(dec)}, unordered {len(free)}: {dict(kinds)}")


if __name__ == "__main__":
    main()
