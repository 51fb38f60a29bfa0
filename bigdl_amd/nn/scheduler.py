"""Data-flow scheduler and loop-frame bookkeeping for DynamicGraph.

Reference: S/nn/Scheduler.scala:36-294 (ready queue, node status, Switch/Merge routing, NextIteration
barriers), S/nn/FrameManager.scala:31-130 (frames of Enter/Exit loops, nodes re-run per iteration).

Node status is one of: absent (not executed in the current iteration), ``READY`` (executed) or ``CONST``
(executed once; a sub-graph fed only by ``Const`` nodes is never re-run, across forwards too). A loop frame
collects the nodes that re-execute every iteration (everything downstream of a ``NextIteration -> Merge``);
``LoopCondition`` arms the frame's barrier with the number of loop variables, each ``NextIteration`` that
arrives counts it down, and when it reaches zero the waiting ``NextIteration`` nodes are released and the
frame's nodes are marked not-executed so the next iteration can run them again.
"""
from collections import deque

READY, CONST = 1, 2


class Frame:
    def __init__(self, name, parent):
        self.name = name
        self.parent = parent
        self.barrier = 0
        self.waiting = []
        self.nodes = []


class FrameManager:
    def __init__(self):
        self.frames = {}
        self.node_frame = {}

    def create(self, name, parent):
        if name not in self.frames:
            self.frames[name] = Frame(name, parent)
        return self.frames[name]

    def _bind(self, node, frame):
        f = self.node_frame.setdefault(node.id, frame)
        if f is not frame:
            raise RuntimeError(f"node {node.element.getName()} cannot be in two frames at the same time")

    def enter(self, node, frame):
        self._bind(node, frame)
        if node not in frame.nodes and self._reexecuted(node, frame):
            frame.nodes.append(node)

    def pend(self, node, frame):
        self._bind(node, frame)
        frame.barrier -= 1
        frame.waiting.append(node)

    @staticmethod
    def _reexecuted(node, frame):
        from .tf import MergeOps, NextIteration

        if isinstance(node.element, MergeOps) and len(node.prevs) == 2 and any(
                isinstance(p.element, NextIteration) for p in node.prevs):
            return True
        return any(p in frame.nodes for p in node.prevs)

    def frame_of(self, node):
        return self.node_frame.get(node.id)


class Scheduler:
    def __init__(self, sources, outputs, executable=None):
        self.sources = list(sources)
        self.outputs = list(outputs)
        self.executable = executable          # optional set of node ids allowed to run
        self.queue = deque()
        self.status = {}
        self.frames = FrameManager()

    def reset(self):
        self.queue.clear()
        self.queue.extend(self.sources)
        self.status = {k: v for k, v in self.status.items() if v == CONST}
        self.frames = FrameManager()

    def executed(self, node):
        return node.id in self.status

    def finished(self):
        if self.queue:
            return False
        for o in self.outputs:
            if not self.executed(o):
                raise RuntimeError(f"output node {o.element.getName()} was not executed")
        return True

    def fetch(self):
        """Next node to run; Const-status nodes and ControlDependency nodes are routed without running."""
        from .tf import ControlDependency

        while self.queue:
            n = self.queue.popleft()
            if isinstance(n.element, ControlDependency) or self.status.get(n.id) == CONST:
                self.schedule(n)
                continue
            return n
        return None

    def schedule(self, node):
        from .tf import Const, Enter, Exit, LoopCondition, NextIteration, SwitchOps, is_random

        e = node.element
        cur = self.frames.frame_of(node)
        if isinstance(e, Enter):
            nxt = self.frames.create(e.frame, cur)
        elif isinstance(e, LoopCondition):
            if cur is None:
                raise RuntimeError("LoopCondition must be inside a loop frame")
            if cur.barrier != 0:
                raise RuntimeError("frame barrier must be 0 when the loop condition runs")
            cur.barrier = len(node.nexts)
            nxt = cur
        elif isinstance(e, NextIteration):
            if cur is None:
                raise RuntimeError("NextIteration must be inside a loop frame")
            nxt = cur
        elif isinstance(e, Exit):
            if cur is None:
                raise RuntimeError("Exit must be inside a loop frame")
            cur.barrier = 0
            nxt = cur.parent
        else:
            nxt = cur

        if self.status.get(node.id) != CONST:
            if not node.prevs:
                self.status[node.id] = CONST if isinstance(e, Const) else READY
            elif all(self.status.get(p.id) == CONST for p in node.prevs) and not is_random(e):
                self.status[node.id] = CONST
            else:
                self.status[node.id] = READY

        cands = self._switch_targets(node) if isinstance(e, SwitchOps) else node.nexts
        self._select(cands, node, nxt)

    @staticmethod
    def _switch_targets(node):
        """Successors on the taken side of a Switch (output slot 1 = false branch, slot 2 = true branch)."""
        both = [n for n, k in zip(node.nexts, node.next_index) if k is None]
        if both:
            raise RuntimeError("a Switch output must be connected through its true or false edge")
        taken = 1 if node.element.output[1] is not None else 2
        out = []
        for n, k in zip(node.nexts, node.next_index):
            if k == taken and n not in out:
                out.append(n)
        return out

    def _ready(self, node):
        from .tf import SwitchOps

        for p in node.prevs:
            if not self.executed(p):
                return False
            if isinstance(p.element, SwitchOps) and node not in self._switch_targets(p):
                return False
        return True

    def _select(self, cands, cur, frame):
        from .tf import MergeOps

        seen = []
        for n in cands:
            if n not in seen:
                seen.append(n)
        for n in seen:
            if self.executable is not None and n.id not in self.executable:
                continue
            if isinstance(n.element, MergeOps):
                if self.executed(n):
                    raise RuntimeError(f"Merge node {n.element.getName()} executed twice in one iteration")
                n.element.setSwitch(n.prevs.index(cur) + 1)
                self._enqueue(n, frame)
            elif self._ready(n):
                self._enqueue(n, frame)

    def _enqueue(self, node, frame):
        from .tf import NextIteration

        if isinstance(node.element, NextIteration):
            if frame is None:
                raise RuntimeError("NextIteration must be inside a loop frame")
            self.frames.pend(node, frame)
            self.status.pop(node.id, None)
            if frame.barrier == 0:
                self._next_iteration(frame)
        else:
            if frame is not None:
                self.frames.enter(node, frame)
            self.queue.append(node)

    def _next_iteration(self, frame):
        from .tf import NextIteration

        self.queue.extend(frame.waiting)
        frame.waiting.clear()
        for n in frame.nodes:
            if not isinstance(n.element, NextIteration):
                self.status.pop(n.id, None)


__all__ = ["Scheduler", "FrameManager", "Frame"]
