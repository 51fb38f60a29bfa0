"""Reference ``bigdl.dataset.base`` helpers (P/dataset/base.py): a console progress bar, a table printer and
``maybe_download``. There is no network here: ``maybe_download`` returns an existing local file and raises with
a clear message otherwise, instead of fetching."""
import os
import sys
import time


class Progbar:
    """Keras-style progress bar: ``update(current, values=[(name, value), ...])``, ``add(n, values)``."""

    def __init__(self, target, width=30, verbose=1, stream=None):
        self.target, self.width, self.verbose = target, width, verbose
        self.stream = stream or sys.stdout
        self.sum_values, self.unique_values = {}, []
        self.seen_so_far, self.start = 0, time.time()

    def update(self, current, values=None, force=False):
        for k, v in values or []:
            if k not in self.sum_values:
                self.sum_values[k] = [v * (current - self.seen_so_far), current - self.seen_so_far]
                self.unique_values.append(k)
            else:
                self.sum_values[k][0] += v * (current - self.seen_so_far)
                self.sum_values[k][1] += current - self.seen_so_far
        self.seen_so_far = current
        if self.verbose:
            frac = min(1.0, current / float(self.target)) if self.target else 1.0
            done = int(self.width * frac)
            bar = "[" + "=" * max(done - 1, 0) + (">" if done < self.width else "=") + "." * (self.width - done) + "]"
            info = " - %ds" % (time.time() - self.start)
            for k in self.unique_values:
                s, n = self.sum_values[k]
                info += " - %s: %.4f" % (k, s / max(n, 1))
            self.stream.write("\r%d/%d %s%s" % (current, self.target, bar, info))
            if current >= self.target:
                self.stream.write("\n")
            self.stream.flush()

    def add(self, n, values=None):
        self.update(self.seen_so_far + n, values)


def display_table(rows, positions):
    """Print ``rows`` (lists of strings) with column ``positions`` (cumulative widths), as the reference does."""
    def line(cells):
        s = ""
        for i, c in enumerate(cells):
            s += str(c)
            s = s[:positions[i]]
            s += " " * (positions[i] - len(s))
        print(s)

    for r in rows:
        line(r)


def maybe_download(filename, work_directory, source_url=None):
    """Path of ``work_directory/filename`` if it exists; downloading is not available in this environment."""
    path = os.path.join(work_directory, filename)
    if os.path.exists(path):
        return path
    raise FileNotFoundError(f"{path} does not exist and this build does not download datasets "
                            f"(source: {source_url}); place the file there first")


__all__ = ["Progbar", "display_table", "maybe_download"]
