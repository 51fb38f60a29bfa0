"""Join rocprofv3 PMC passes (one counter set per run) into one per-kernel table.

    python tools/pmc_table.py gpurun_out/pmc_1/run_results.db gpurun_out/pmc_2/run_results.db ... [--top 12]

Per kernel name: calls, mean duration (us, from the PMC runs), mean FETCH_SIZE / WRITE_SIZE (KB per call),
the implied HBM GB/s ((FETCH + WRITE) * 1024 / duration; gfx950's FETCH_SIZE can under-count wide coalesced
reads by up to 2x — cdna_hip_programming.md §7 — so this is a LOWER bound), and the MFMA-busy fraction
SQ_VALU_MFMA_BUSY_CYCLES / (4 SIMDs x SQ_BUSY_CU_CYCLES) when those counters were collected."""
import argparse
import sqlite3
from collections import defaultdict


def load(db):
    c = sqlite3.connect(db)
    rows = c.execute("select kernel_name, counter_name, value, duration, dispatch_id from counters_collection")
    return rows.fetchall()


def short(n):
    n = n.replace("(anonymous namespace)::", "")
    if n.startswith("void "):
        n = n[5:]
    i = n.find("(")
    return (n[:i] if i > 0 else n)[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dbs", nargs="+")
    ap.add_argument("--top", type=int, default=12)
    a = ap.parse_args()
    val = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    calls = defaultdict(set)
    for db in a.dbs:
        for k, cn, v, d, did in load(db):
            key = short(k)
            val[key][cn].append(v)
            if cn in ("FETCH_SIZE", "GRBM_GUI_ACTIVE", "SQ_WAVE_CYCLES"):
                dur[key].append(d)
            calls[key].add((db, did))
    tot = {k: sum(v) / max(1, len(v)) * len(v) for k, v in dur.items()}
    order = sorted(tot, key=lambda k: -tot[k])[:a.top]
    print(f"{'kernel':70s} {'calls':>5s} {'us/call':>8s} {'FETCH KB':>10s} {'WRITE KB':>10s} {'GB/s>=':>8s} "
          f"{'MFMA busy':>9s}")
    for k in order:
        m = lambda cn: (sum(val[k][cn]) / len(val[k][cn])) if val[k].get(cn) else float("nan")  # noqa: E731
        us = sum(dur[k]) / len(dur[k]) / 1e3
        f, w = m("FETCH_SIZE"), m("WRITE_SIZE")
        gbs = (f + w) * 1024 / (us * 1e3) if us > 0 else float("nan")
        busy = m("SQ_VALU_MFMA_BUSY_CYCLES") / (4 * m("SQ_BUSY_CU_CYCLES")) if val[k].get("SQ_BUSY_CU_CYCLES") \
            else float("nan")
        print(f"{k:70s} {len(dur[k]):5d} {us:8.1f} {f:10.0f} {w:10.0f} {gbs:8.0f} {busy:9.3f}")


if __name__ == "__main__":
    main()
