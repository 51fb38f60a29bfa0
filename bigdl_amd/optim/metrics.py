"""Per-iteration timing counters (reference S/optim/Metrics.scala:31-123)."""
import time
from collections import defaultdict


class Metrics:
    def __init__(self):
        self._sum = defaultdict(float)
        self._cnt = defaultdict(int)

    def add(self, name, value):
        self._sum[name] += value
        self._cnt[name] += 1
        return self

    def set(self, name, value):
        self._sum[name] = value
        self._cnt[name] = 1
        return self

    def get(self, name):
        c = self._cnt.get(name, 0)
        return (self._sum[name] / c) if c else 0.0

    def reset(self):
        self._sum.clear()
        self._cnt.clear()

    def summary(self, unit="s", scale=1.0):
        lines = ["========== Metrics Summary =========="]
        for k in sorted(self._sum):
            lines.append(f"{k} : {self._sum[k] * scale / max(self._cnt[k], 1):.6f} {unit}")
        lines.append("=====================================")
        return "\n".join(lines)


class Timer:
    def __init__(self, metrics, name):
        self.metrics, self.name = metrics, name

    def __enter__(self):
        self.t0 = time.perf_counter()
        return self

    def __exit__(self, *a):
        self.metrics.add(self.name, time.perf_counter() - self.t0)
