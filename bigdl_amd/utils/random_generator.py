"""Random number generation (reference: S/utils/RandomGenerator.scala:23-272, MT19937 ``RNG``).

The reference keeps a per-thread Mersenne Twister used by init methods, dropout and shuffling. Here the
host generator is a seeded ``torch.Generator`` (MT19937 on CPU as well), and device-side randomness
(dropout masks) uses the device generator seeded from it, so ``RNG.setSeed(s)`` makes a whole run
reproducible.
"""
import math

import torch


class RandomGenerator:
    def __init__(self, seed=None):
        self._gen = torch.Generator()
        self.setSeed(seed if seed is not None else 1)

    def setSeed(self, seed):
        self._seed = int(seed)
        self._gen.manual_seed(self._seed)
        torch.manual_seed(self._seed)
        return self

    def getSeed(self):
        return self._seed

    @property
    def generator(self):
        return self._gen

    def uniform(self, a=0.0, b=1.0, size=None):
        if size is None:
            return a + (b - a) * torch.rand((), generator=self._gen).item()
        return a + (b - a) * torch.rand(size, generator=self._gen)

    def normal(self, mean=0.0, std=1.0, size=None):
        if size is None:
            return mean + std * torch.randn((), generator=self._gen).item()
        return mean + std * torch.randn(size, generator=self._gen)

    def bernoulli(self, p, size=None):
        if size is None:
            return float(torch.rand((), generator=self._gen).item() < p)
        return (torch.rand(size, generator=self._gen) < p).float()

    def exponential(self, lam=1.0):
        u = torch.rand((), generator=self._gen).item()
        return -math.log(1 - u) / lam

    def randperm(self, n):
        return torch.randperm(n, generator=self._gen)

    def random(self):
        return int(torch.randint(0, 2 ** 31 - 1, (), generator=self._gen).item())

    def clone(self):
        r = RandomGenerator(self._seed)
        r._gen.set_state(self._gen.get_state())
        return r


RNG = RandomGenerator()
