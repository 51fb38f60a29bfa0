"""Summarize rocprofv3 rocpd SQLite output: per-kernel time table and per-kernel PMC counter averages."""
import sqlite3
import sys


def kernels(db, top=30, skip_first=0, after=None, per=1):
    """Per-kernel totals. ``after=(substr, k)``: only dispatches that start after the k-th dispatch of a kernel whose
    name contains substr (e.g. the once-per-step input kernel: skip setup / warm-up); totals are divided by ``per``
    (the number of steps left) to give per-step times."""
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name_col = "kernel_name" if "kernel_name" in cols else ("name" if "name" in cols else None)
    rows = c.execute(f"select {name_col}, start, end from kernels order by start").fetchall()
    if after is not None:
        marks = [s for n, s, _ in rows if after[0] in n]
        if len(marks) > after[1]:
            t0 = marks[after[1]]
            rows = [r for r in rows if r[1] >= t0]
    agg = {}
    for n, s, e in rows:
        a = agg.setdefault(n, [0, 0.0])
        a[0] += 1
        a[1] += (e - s) / 1e6
    for a in agg.values():
        a[1] /= per
    tot = sum(v[1] for v in agg.values())
    unit = "ms" if per == 1 else "ms/step"
    out = [f"total kernel time {tot:.3f} {unit} over {len(rows)} dispatches" + (f" ({per} steps)" if per > 1 else "")]
    for n, (cnt, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        out.append(f"{ms:9.3f} {unit} {100 * ms / tot:5.1f}% {cnt:6d}  {n[:150]}")
    return "\n".join(out)


def counters(db):
    c = sqlite3.connect(db)
    try:
        rows = c.execute("select * from counters_collection").fetchall()
        cols = [d[0] for d in c.execute("select * from counters_collection").description]
    except sqlite3.Error as e:
        return f"no counters: {e}"
    ki = cols.index("kernel_name") if "kernel_name" in cols else None
    ci = cols.index("counter_name")
    vi = cols.index("value")
    di = cols.index("dispatch_id") if "dispatch_id" in cols else None
    agg = {}
    for r in rows:
        k = (r[ki][:110] if ki is not None else "?", r[ci])
        agg.setdefault(k, []).append(r[vi])
    out = []
    for (k, cn), vs in sorted(agg.items()):
        out.append(f"{k} | {cn} = {sum(vs) / len(vs):.4g} (n={len(vs)})")
    return "\n".join(out)


if __name__ == "__main__":
    # kernels DB [MARK K STEPS]: per-step table of the dispatches after the K-th dispatch of kernel MARK
    mode, db = sys.argv[1], sys.argv[2]
    if mode == "kernels" and len(sys.argv) >= 6:
        print(kernels(db, after=(sys.argv[3], int(sys.argv[4])), per=int(sys.argv[5])))
    else:
        print(kernels(db) if mode == "kernels" else counters(db))
