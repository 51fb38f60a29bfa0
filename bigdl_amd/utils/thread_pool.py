"""Host task pool (reference S/utils/ThreadPool.scala:38-270: invokeAndWait :130, invokeAndWait2 with timeout and
cancellation :156-164 used for straggler dropping, invoke :201/:218, sync, setMKLThread :89).

GPU work is issued on HIP streams; this pool runs host-side tasks (data preparation, per-replica bookkeeping,
checkpoint I/O). Native batch assembly runs on the C++ pool in csrc/host_runtime.cpp instead.
"""
import concurrent.futures as cf
import threading


class ThreadPool:
    def __init__(self, poolSize):
        self.poolSize = int(poolSize)
        self._pool = cf.ThreadPoolExecutor(max_workers=max(1, self.poolSize), thread_name_prefix="bigdl")
        self._lock = threading.Lock()

    def getPoolSize(self):
        return self.poolSize

    def setPoolSize(self, n):
        """Recreate the pool with ``n`` workers (ThreadPool.setPoolSize)."""
        with self._lock:
            if n != self.poolSize:
                self._pool.shutdown(wait=True)
                self.poolSize = int(n)
                self._pool = cf.ThreadPoolExecutor(max_workers=max(1, self.poolSize), thread_name_prefix="bigdl")
        return self

    def setMKLThread(self, n):
        """No MKL on the GPU engine; kept for API parity."""
        return self

    def invoke(self, tasks):
        """Submit callables (or one callable) and return the futures without waiting."""
        if callable(tasks):
            return self._pool.submit(tasks)
        return [self._pool.submit(t) for t in tasks]

    def invokeAndWait(self, tasks, timeout=None):
        """Run all tasks and return their results in order (raises the first task error)."""
        futs = [self._pool.submit(t) for t in tasks]
        return [f.result(timeout=timeout) for f in futs]

    def invokeAndWait2(self, tasks, timeout=None):
        """Run tasks with a deadline; returns the futures: finished ones hold results, the others are cancelled
        (the reference drops straggler replicas this way, DistriOptimizer.scala:278)."""
        futs = [self._pool.submit(t) for t in tasks]
        done, pending = cf.wait(futs, timeout=timeout)
        for f in pending:
            f.cancel()
        return futs

    def sync(self, futures, timeout=None):
        for f in futures:
            f.result(timeout=timeout)

    def shutdown(self):
        self._pool.shutdown(wait=True)


__all__ = ["ThreadPool"]
