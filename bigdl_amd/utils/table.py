"""Lua-style heterogeneous table (reference: S/utils/Table.scala:34, factory ``T(...)`` :323).

Keys are usually 1-based integers (multi-input activities) or strings (optimizer state). A Table is also
an ``Activity`` — modules that take several inputs (CAddTable, JoinTable, ParallelTable…) take a Table.
"""


class Table:
    __slots__ = ("_state", "_top")

    def __init__(self, *values, **kv):
        self._state = {}
        self._top = 0
        for v in values:
            self.insert(v)
        for k, v in kv.items():
            self._state[k] = v

    # -- access ---------------------------------------------------------------------------------
    def __getitem__(self, k):
        return self._state[k]

    def __setitem__(self, k, v):
        self._state[k] = v
        if isinstance(k, int) and k > self._top:
            self._top = k

    def __delitem__(self, k):
        del self._state[k]

    def __contains__(self, k):
        return k in self._state

    def get(self, k, default=None):
        return self._state.get(k, default)

    def getOrElse(self, k, default):
        return self._state.get(k, default)

    def contains(self, k):
        return k in self._state

    def apply(self, k):
        return self._state[k]

    def update(self, k, v):
        self[k] = v
        return self

    def insert(self, *args):
        """insert(value) appends at length+1; insert(index, value) shifts like Lua table.insert."""
        if len(args) == 1:
            self._top = self.length() + 1
            self._state[self._top] = args[0]
        else:
            idx, v = args
            n = self.length()
            for i in range(n, idx - 1, -1):
                self._state[i + 1] = self._state[i]
            self._state[idx] = v
            self._top = max(self._top, n + 1)
        return self

    def remove(self, idx=None):
        n = self.length()
        if n == 0:
            return None
        if idx is None:
            idx = n
        v = self._state.pop(idx, None)
        for i in range(idx, n):
            self._state[i] = self._state.pop(i + 1)
        self._top = n - 1
        return v

    def length(self):
        n = 0
        while (n + 1) in self._state:
            n += 1
        return n

    def __len__(self):
        return self.length()

    def keys(self):
        return list(self._state.keys())

    def values(self):
        return list(self._state.values())

    def items(self):
        return list(self._state.items())

    def clear(self):
        self._state.clear()
        self._top = 0
        return self

    def toSeq(self):
        return [self._state[i] for i in range(1, self.length() + 1)]

    def __iter__(self):
        return iter(self.toSeq())

    def clone(self):
        t = Table()
        for k, v in self._state.items():
            t._state[k] = v.clone() if hasattr(v, "clone") else v
        t._top = self._top
        return t

    def __eq__(self, other):
        if not isinstance(other, Table) or set(self._state) != set(other._state):
            return False
        import torch

        for k, v in self._state.items():
            o = other._state[k]
            if isinstance(v, torch.Tensor):
                if not (isinstance(o, torch.Tensor) and v.shape == o.shape and torch.equal(v, o)):
                    return False
            elif v != o:
                return False
        return True

    def __repr__(self):
        inner = ", ".join(f"{k}: {_short(v)}" for k, v in self._state.items())
        return "{" + inner + "}"

    # torch-like helpers used when tables carry tensors
    def to(self, *args, **kw):
        t = Table()
        for k, v in self._state.items():
            t._state[k] = v.to(*args, **kw) if hasattr(v, "to") else v
        t._top = self._top
        return t


def _short(v):
    import torch

    if isinstance(v, torch.Tensor):
        return f"Tensor{tuple(v.shape)}"
    return repr(v)


def T(*values, **kv):
    """Reference factory ``T(a, b, c)`` → 1-based Table."""
    return Table(*values, **kv)
