"""Print every PMC counter of one or more rocprofv3 --pmc databases, averaged per dispatch, per kernel.

    python tools/pmc_dump.py gpurun_out/pmcl/p1/run_results.db [...] [--match conv_nt]
"""
import argparse
import sqlite3
from collections import defaultdict


def short(n):
    n = n.replace("(anonymous namespace)::", "")
    if n.startswith("void "):
        n = n[5:]
    i = n.find("(")
    return (n[:i] if i > 0 else n)[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dbs", nargs="+")
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    val = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    for db in a.dbs:
        c = sqlite3.connect(db)
        for k, cn, v, d in c.execute("select kernel_name, counter_name, value, duration from counters_collection"):
            key = short(k)
            if a.match and a.match not in key:
                continue
            val[key][cn].append(v)
            dur[key].append(d)
    for k in sorted(val, key=lambda k: -sum(dur[k])):
        print(f"{k}  (~{sum(dur[k]) / len(dur[k]) / 1e3:.1f} us/dispatch)")
        for cn in sorted(val[k]):
            vs = val[k][cn]
            print(f"    {cn:32s} {sum(vs) / len(vs):16.1f}")


if __name__ == "__main__":
    main()
