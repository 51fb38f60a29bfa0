"""Tree-structured LSTMs.

Reference: S/nn/TreeLSTM.scala:27-60 (base: input / hidden sizes, shared parameters across node cells),
S/nn/BinaryTreeLSTM.scala:33-573 (binary constituency Tree-LSTM, Tai et al. 2015: leaf module c = W_c x,
h = sigmoid(W_o x) * tanh(c); composer gates i, f_l, f_r, u, o from (h_l, h_r); TensorTree encoding of trees).

MI355X design: the reference clones a leaf / composer module per tree node and recurses node by node. Here the
whole batch of trees is evaluated level-synchronously: all leaves in one GEMM, then one GEMM per tree level over
every composer node of every tree in the batch whose children are ready, so the number of kernel launches is
O(tree height) instead of O(nodes). The gate weights of the five composer gates are stacked into one
(5H x H) matrix per child, so each level is two GEMMs + one fused pointwise pass. Backward is torch autograd
over the same level schedule.

Tree encoding (TensorTree): ``trees`` is (batch, nodes, k); row n = [child_1, child_2, ..., tag] with 1-based
child node indices (0 = none), last column = -1 for the root or the 1-based leaf (word) index for leaves;
``child_1 == -1`` marks a padding row.
"""
import math

import torch

from ..utils.table import Table
from .abstractnn import AutogradModule
from .init_methods import RandomUniform



def _lin(x, w, b=None):
    """x w^T (+ b): the native MFMA GEMM on the GPU engine (ops/conv_fn.linear), torch.addmm on the CPU."""
    if x.is_cuda:
        from ..ops import conv_fn

        return conv_fn.linear(x.float(), w.float(), None if b is None else b.float())
    return torch.addmm(b, x, w.t()) if b is not None else x @ w.t()

class TensorTree:
    """1-based view of one tree encoding (reference BinaryTreeLSTM.scala TensorTree)."""

    def __init__(self, content):
        self.content = content
        self.c = content.long().tolist() if isinstance(content, torch.Tensor) else [list(map(int, r)) for r in content]

    @property
    def nodeNumber(self):
        return len(self.c)

    def children(self, index):
        return self.c[index - 1][:-1]

    def getRoot(self):
        for i, row in enumerate(self.c):
            if row[-1] == -1:
                return i + 1
        raise RuntimeError("There is no root in the tensor tree")

    def leafIndex(self, index):
        return self.c[index - 1][-1]

    def hasChild(self, index):
        return self.c[index - 1][0] > 0

    def noChild(self, index):
        return self.c[index - 1][0] == 0

    def isPadding(self, index):
        return self.c[index - 1][0] == -1

    def addChild(self, parent, child):
        for i in range(len(self.c[parent - 1]) - 1):
            if self.c[parent - 1][i] == 0:
                self.c[parent - 1][i] = int(child)
                if isinstance(self.content, torch.Tensor):
                    self.content[parent - 1, i] = child
                return

    def markAsRoot(self, index):
        self.c[index - 1][-1] = -1
        if isinstance(self.content, torch.Tensor):
            self.content[index - 1, -1] = -1

    def markAsLeaf(self, index, leafIndex):
        self.c[index - 1][-1] = int(leafIndex)
        if isinstance(self.content, torch.Tensor):
            self.content[index - 1, -1] = leafIndex


class TreeLSTM(AutogradModule):
    """Base class (reference TreeLSTM.scala:27)."""

    def __init__(self, inputSize, hiddenSize=150):
        super().__init__()
        self.inputSize, self.hiddenSize = inputSize, hiddenSize


class BinaryTreeLSTM(TreeLSTM):
    """Binary Tree-LSTM. Input Table(inputs (B, L, inputSize), trees (B, N, 3)); output (B, N, hiddenSize) with
    the hidden state of every tree node (zeros for padding rows)."""

    def __init__(self, inputSize, hiddenSize, gateOutput=True, withGraph=True):
        super().__init__(inputSize, hiddenSize)
        self.gateOutput, self.withGraph = gateOutput, withGraph
        H = hiddenSize
        ng = 5 if gateOutput else 4
        nl = 2 if gateOutput else 1
        self.register_parameter("leafWeight", "leafGradWeight", torch.empty(nl * H, inputSize))
        self.register_parameter("leafBias", "leafGradBias", torch.empty(nl * H))
        self.register_parameter("leftWeight", "leftGradWeight", torch.empty(ng * H, H))
        self.register_parameter("leftBias", "leftGradBias", torch.empty(ng * H))
        self.register_parameter("rightWeight", "rightGradWeight", torch.empty(ng * H, H))
        self.register_parameter("rightBias", "rightGradBias", torch.empty(ng * H))
        self.reset()

    def reset(self):
        with torch.no_grad():
            a = 1.0 / math.sqrt(self.inputSize)
            b = 1.0 / math.sqrt(self.hiddenSize)
            for name, s in (("leafWeight", a), ("leafBias", a), ("leftWeight", b), ("leftBias", b),
                            ("rightWeight", b), ("rightBias", b)):
                RandomUniform(-s, s).init(getattr(self, name))

    # ------------------------------------------------------------------------------------ schedule
    @staticmethod
    def _schedule(trees):
        """Per-tree node lists grouped by height: leaves [(b, n, leafIdx)], levels [[(b, n, l, r)]]."""
        leaves, levels = [], {}
        for b in range(trees.shape[0]):
            t = TensorTree(trees[b])
            height = {}

            def h(n):
                if n in height:
                    return height[n]
                if t.noChild(n):
                    leaves.append((b, n - 1, t.leafIndex(n) - 1))
                    height[n] = 0
                    return 0
                l, r = t.children(n)[0], t.children(n)[1]
                v = 1 + max(h(l), h(r))
                height[n] = v
                levels.setdefault(v, []).append((b, n - 1, l - 1, r - 1))
                return v

            h(t.getRoot())
        return leaves, [levels[k] for k in sorted(levels)]

    def fn(self, x):
        inputs, trees = x[1], x[2]
        B, N = trees.shape[0], trees.shape[1]
        H = self.hiddenSize
        dev = inputs.device
        leaves, levels = self._schedule(trees.detach().cpu())
        zeros = inputs.new_zeros(B * N, H)
        C, Hs = zeros, zeros
        if leaves:
            lb = torch.tensor([b for b, _, _ in leaves], device=dev)
            ln = torch.tensor([b * N + n for b, n, _ in leaves], device=dev)
            li = torch.tensor([i for _, _, i in leaves], device=dev)
            xin = inputs[lb, li]
            g = _lin(xin, self.leafWeight, self.leafBias)
            c = g[:, :H]
            h = torch.sigmoid(g[:, H:]) * torch.tanh(c) if self.gateOutput else torch.tanh(c)
            C = C.index_copy(0, ln, c)
            Hs = Hs.index_copy(0, ln, h)
        bias = self.leftBias + self.rightBias
        for lvl in levels:
            node = torch.tensor([b * N + n for b, n, _, _ in lvl], device=dev)
            left = torch.tensor([b * N + l for b, _, l, _ in lvl], device=dev)
            right = torch.tensor([b * N + r for b, _, _, r in lvl], device=dev)
            lh, rh, lc, rc = Hs[left], Hs[right], C[left], C[right]
            g = _lin(lh, self.leftWeight, bias) + _lin(rh, self.rightWeight)
            i = torch.sigmoid(g[:, :H])
            lf = torch.sigmoid(g[:, H:2 * H])
            rf = torch.sigmoid(g[:, 2 * H:3 * H])
            u = torch.tanh(g[:, 3 * H:4 * H])
            c = i * u + lf * lc + rf * rc
            h = torch.sigmoid(g[:, 4 * H:]) * torch.tanh(c) if self.gateOutput else torch.tanh(c)
            C = C.index_copy(0, node, c)
            Hs = Hs.index_copy(0, node, h)
        return Hs.reshape(B, N, H)

    def updateGradInput(self, input, gradOutput):
        gi = super().updateGradInput(input, gradOutput)
        return Table(gi[1], torch.zeros_like(input[2]))

    def __repr__(self):
        return f"BinaryTreeLSTM({self.inputSize}, {self.hiddenSize}, gateOutput={self.gateOutput})"


__all__ = ["TensorTree", "TreeLSTM", "BinaryTreeLSTM"]
