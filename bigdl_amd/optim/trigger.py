"""Triggers evaluated on the driver state table (reference S/optim/Trigger.scala:26-155).

State keys: "epoch" (1-based), "neval" (1-based iteration counter), "Loss", "score",
"recordsProcessedThisEpoch".
"""


class Trigger:
    def __call__(self, state):
        raise NotImplementedError

    def __and__(self, other):
        return And(self, other)

    def __or__(self, other):
        return Or(self, other)

    @staticmethod
    def everyEpoch():
        return EveryEpoch()

    @staticmethod
    def severalIteration(interval):
        return SeveralIteration(interval)

    @staticmethod
    def maxEpoch(m):
        return MaxEpoch(m)

    @staticmethod
    def maxIteration(m):
        return MaxIteration(m)

    @staticmethod
    def maxScore(m):
        return MaxScore(m)

    @staticmethod
    def minLoss(m):
        return MinLoss(m)

    @staticmethod
    def and_(first, *others):
        return And(first, *others)

    @staticmethod
    def or_(first, *others):
        return Or(first, *others)


class EveryEpoch(Trigger):
    def __init__(self):
        self.last = -1

    def __call__(self, state):
        e = state.get("epoch")
        if self.last == -1:
            self.last = e
            return False
        if e > self.last:
            self.last = e
            return True
        return False


class SeveralIteration(Trigger):
    def __init__(self, interval):
        self.interval = interval

    def __call__(self, state):
        n = state.get("neval")
        return n != 0 and (n - 1) % self.interval == 0 and n > 1


class MaxEpoch(Trigger):
    def __init__(self, m):
        self.max = m

    def __call__(self, state):
        return state.get("epoch") > self.max


class MaxIteration(Trigger):
    def __init__(self, m):
        self.max = m

    def __call__(self, state):
        return state.get("neval") > self.max


class MaxScore(Trigger):
    def __init__(self, m):
        self.max = m

    def __call__(self, state):
        s = state.get("score")
        return s is not None and s > self.max


class MinLoss(Trigger):
    def __init__(self, m):
        self.min = m

    def __call__(self, state):
        l = state.get("Loss")
        return l is not None and l < self.min


class And(Trigger):
    def __init__(self, *ts):
        self.ts = ts

    def __call__(self, state):
        return all(t(state) for t in self.ts)


class Or(Trigger):
    def __init__(self, *ts):
        self.ts = ts

    def __call__(self, state):
        return any(t(state) for t in self.ts)


everyEpoch = Trigger.everyEpoch
severalIteration = Trigger.severalIteration
maxEpoch = Trigger.maxEpoch
maxIteration = Trigger.maxIteration
maxScore = Trigger.maxScore
minLoss = Trigger.minLoss
