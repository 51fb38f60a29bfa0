"""Per-stream busy time, overlap and idle gaps of a rocprofv3 kernel trace (rocpd SQLite), over the dispatches after the
k-th dispatch of a marker kernel: how much of the wall the GPU had at least one kernel, and how much two streams ran
concurrently.  usage: rocpd_streams.py DB MARKER K STEPS"""
import sqlite3
import sys


def union(iv):
    iv = sorted(iv)
    tot, cur_s, cur_e = 0, None, None
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main(db, marker, k, steps):
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end, stream_id, queue_id from kernels order by start").fetchall()
    marks = [s for n, s, _, _, _ in rows if marker in n]
    t0 = marks[k]
    rows = [r for r in rows if r[1] >= t0]
    t1 = max(r[2] for r in rows)
    wall = (t1 - t0) / 1e6 / steps
    by = {}
    for n, s, e, sid, qid in rows:
        by.setdefault((sid, qid), []).append((s, e))
    print(f"wall {wall:.3f} ms/step, GPU busy (union) {union([(s, e) for _, s, e, _, _ in rows]) / 1e6 / steps:.3f} ms/step")
    for key, iv in sorted(by.items(), key=lambda kv: -len(kv[1])):
        print(f"stream {key}: {len(iv) // steps} dispatches/step, busy {union(iv) / 1e6 / steps:.3f} ms/step")
    keys = list(by)
    if len(keys) >= 2:
        a, b = by[keys[0]], by[keys[1]]
        both = union(a) + union(b) - union(a + b)
        print(f"both of the two busiest streams running: {both / 1e6 / steps:.3f} ms/step")
    # per-kernel time on each of the two busiest streams (the compute stream is the step's critical path)
    for key in sorted(by, key=lambda kk: -len(by[kk]))[:2]:
        agg = {}
        for n, s, e, sid, qid in rows:
            if (sid, qid) == key:
                a = agg.setdefault(n, [0, 0.0])
                a[0] += 1
                a[1] += (e - s) / 1e6 / steps
        print(f"-- stream {key} kernels (ms/step, dispatches/step)")
        for n, (cnt, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:25]:
            print(f"{ms:8.3f} {cnt / steps:6.1f}  {n[:120]}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]))
