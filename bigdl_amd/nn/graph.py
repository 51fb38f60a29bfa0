"""Graph models: ``Graph(inputs, outputs)`` over module nodes.

Reference: S/nn/Graph.scala:72 (factories :476-560, stopGradient :248), StaticGraph.scala:38 (topological
forward :56-67, backward :82-103), DynamicGraph.scala, utils/DirectedGraph.scala:36 (topological sort).

Build with ``node = Layer(...).inputs(prev_node, ...)`` (or ``Layer(...)(prev)``); a node with several
predecessors receives a 1-based Table of their outputs in edge order. Execution follows a topological
order computed once; backward walks it in reverse, summing gradients at fan-out nodes.
"""

import torch

from ..utils.table import Table
from .abstractnn import AbstractModule, _t_begin, _t_end
from .activation import Identity
from .containers import Container, add_activity


class Node:
    _ids = 0

    def __init__(self, element):
        self.element = element
        self.prevs = []
        self.nexts = []
        self.prev_index = []     # per incoming edge: None, or the 1-based slot of the predecessor's output Table
        self.next_index = []     # the same edge seen from the predecessor
        Node._ids += 1
        self.id = Node._ids

    def add_next(self, node, from_index=None):
        """Edge ``self -> node``; ``from_index`` selects one entry of this node's Table output
        (reference utils/DirectedGraph.scala Edge(fromIndex))."""
        self.nexts.append(node)
        self.next_index.append(from_index)
        node.prevs.append(self)
        node.prev_index.append(from_index)
        return node

    def remove_prev(self, prev):
        while prev in self.prevs:
            i = self.prevs.index(prev)
            del self.prevs[i], self.prev_index[i]
        while self in prev.nexts:
            j = prev.nexts.index(self)
            del prev.nexts[j], prev.next_index[j]

    def __rshift__(self, node):
        return self.add_next(node)

    def setName(self, name):
        self.element.setName(name)
        return self

    def __repr__(self):
        return f"Node({self.element!r})"


def Input(name=None):
    """A graph input placeholder node."""
    m = Identity()
    if name:
        m.setName(name)
    node = Node(m)
    node._is_input = True
    return node


def topo_sort(outputs):
    order, seen, temp = [], set(), set()

    def visit(n):
        if n.id in seen:
            return
        if n.id in temp:
            raise ValueError("Graph has a cycle")
        temp.add(n.id)
        for p in n.prevs:
            visit(p)
        temp.discard(n.id)
        seen.add(n.id)
        order.append(n)

    for o in outputs:
        visit(o)
    return order


def edge_value(out, from_index):
    return out if from_index is None else out[from_index]


def add_edge_grad(acc, g, from_index):
    """Accumulate the gradient arriving over one edge; an indexed edge contributes to one Table slot."""
    if from_index is None:
        return add_activity(acc, g)
    acc = acc if acc is not None else Table()
    acc[from_index] = add_activity(acc.get(from_index), g)
    return acc


class Graph(Container):
    """Static DAG model (reference StaticGraph)."""

    def __init__(self, inputs, outputs, variables=None):
        inputs = list(inputs) if isinstance(inputs, (list, tuple)) else [inputs]
        outputs = list(outputs) if isinstance(outputs, (list, tuple)) else [outputs]
        super().__init__()
        self.inputs_nodes = inputs
        self.output_nodes = outputs
        self.order = topo_sort(outputs)
        for n in inputs:
            if n not in self.order:
                self.order.insert(0, n)
        self.modules = [n.element for n in self.order]
        self._stop_grad = set()

    def getInputs(self):
        return self.inputs_nodes

    def getOutputs(self):
        return self.output_nodes

    def node(self, name):
        for n in self.order:
            if n.element.hasName() and n.element.getName() == name:
                return n
        raise KeyError(name)

    def stopGradient(self, names):
        self._stop_grad |= set(names)
        return self

    def _node_input(self, n, outs, graph_input):
        if n in self.inputs_nodes and not n.prevs:
            if len(self.inputs_nodes) == 1:
                return graph_input
            return graph_input[self.inputs_nodes.index(n) + 1]
        vals = [edge_value(outs[p.id], k) for p, k in zip(n.prevs, n.prev_index)]
        if len(vals) == 1:
            return vals[0]
        t = Table()
        for i, v in enumerate(vals):
            t[i + 1] = v
        return t

    def updateOutput(self, input):
        outs = {}
        self._node_inputs = {}
        for n in self.order:
            x = self._node_input(n, outs, input)
            self._node_inputs[n.id] = x
            pre = getattr(n, "fuse_pre", None)   # inference fusion hook (nn.fusion.fuse_graph_for_inference)
            if pre is not None:
                pre(outs, x)
            # training residual fusion (nn.fusion._fuse_graph_training): this BN adds the shortcut node's output
            # (and applies the ReLU) in its own pass; the CAddTable after it only passes that result on
            rs = getattr(n, "res_src", None)
            if rs is not None:
                n.element._graph_residual = outs[rs.id]
            pi = getattr(n, "pass_index", None)
            if pi is not None:
                outs[n.id] = x[pi]
                continue
            run = getattr(n, "fuse_run", None)   # planned runner (quantized.int8_graph) replacing forward
            outs[n.id] = run(x) if run is not None else n.element.forward(x)
        self._outs = outs
        if len(self.output_nodes) == 1:
            return outs[self.output_nodes[0].id]
        t = Table()
        for i, o in enumerate(self.output_nodes):
            t[i + 1] = outs[o.id]
        return t

    def _run_backward(self, input, gradOutput, acc_params, upd_input):
        grads = {}
        if len(self.output_nodes) == 1:
            grads[self.output_nodes[0].id] = gradOutput
        else:
            for i, o in enumerate(self.output_nodes):
                grads[o.id] = add_activity(grads.get(o.id), gradOutput[i + 1])
        gin = None
        for n in reversed(self.order):
            g = grads.get(n.id)
            if g is None:
                continue
            x = self._node_inputs[n.id]
            m = n.element
            pi = getattr(n, "pass_index", None)
            if pi is not None:           # fused residual add: the BN producing input ``pi`` owns the ReLU mask
                p = n.prevs[pi - 1]
                grads[p.id] = add_edge_grad(grads.get(p.id), g, None)
                continue
            folded = self._fold_fanout(n, m, x, grads) if upd_input else False
            if acc_params and upd_input:
                gi = m.backward(x, g)
            elif upd_input:
                gi = m.updateGradInput(x, g)
            else:
                m.accGradParameters(x, g)
                gi = m.gradInput
            rs = getattr(n, "res_src", None)
            if rs is not None:           # the shortcut's gradient: the ReLU-masked output gradient of the fused BN
                d = m.__dict__.pop("_dres", None)
                if d is None:
                    d = g * (m.output > 0).to(g.dtype)
                grads[rs.id] = add_edge_grad(grads.get(rs.id), d, None)
            if m.hasName() and m.getName() in self._stop_grad:
                continue
            if folded:                   # gi already holds the sum over every consumer of the input
                grads[n.prevs[0].id] = gi
                continue
            if n in self.inputs_nodes:
                if len(self.inputs_nodes) == 1:
                    gin = add_activity(gin, gi)
                else:
                    gin = gin if gin is not None else Table()
                    k = self.inputs_nodes.index(n) + 1
                    gin[k] = add_activity(gin.get(k), gi)
                continue
            if len(n.prevs) == 1:
                p = n.prevs[0]
                grads[p.id] = add_edge_grad(grads.get(p.id), gi, n.prev_index[0])
            else:
                for i, p in enumerate(n.prevs):
                    grads[p.id] = add_edge_grad(grads.get(p.id), gi[i + 1] if gi is not None else None,
                                                n.prev_index[i])
        return gin

    @staticmethod
    def _fold_fanout(n, m, x, grads):
        """A conv that is the last consumer (in backward order) of a fanned-out tensor sums the gradient the other
        consumers already produced inside its data-gradient epilogue instead of a separate add pass (planned by
        nn.fusion._fuse_graph_training as ``node.fold_fanout``)."""
        if not getattr(n, "fold_fanout", False):
            return False
        acc = grads.get(n.prevs[0].id)
        if not (isinstance(acc, torch.Tensor) and isinstance(x, torch.Tensor) and acc.is_cuda
                and acc.dtype == x.dtype and acc.shape == x.shape
                and acc.is_contiguous(memory_format=torch.channels_last)):
            return False
        m._dgrad_addend = acc
        # the result is the input's complete gradient: a BN that produced it may reduce in this epilogue
        m._dgrad_bn_once = n.fold_bn
        return True

    def backward(self, input, gradOutput):
        t0 = _t_begin(gradOutput)
        self.gradInput = self._run_backward(input, gradOutput, True, True)
        _t_end(self, t0, "backward_time")
        return self.gradInput

    def updateGradInput(self, input, gradOutput):
        return self._run_backward(input, gradOutput, False, True)

    def accGradParameters(self, input, gradOutput):
        self._run_backward(input, gradOutput, True, False)

    def saveGraphTopology(self, logPath):
        import json
        import os

        os.makedirs(logPath, exist_ok=True)
        desc = [{"id": n.id, "module": repr(n.element), "prevs": [p.id for p in n.prevs]} for n in self.order]
        with open(os.path.join(logPath, "graph.json"), "w") as f:
            json.dump(desc, f, indent=1)
        return self

    def __repr__(self):
        return f"Graph({len(self.order)} nodes)"


    @staticmethod
    def dynamic(inputs, outputs, variables=None, generateBackward=True):
        """Reference Graph.dynamic (S/nn/Graph.scala:540): a DynamicGraph run by the Scheduler."""
        return DynamicGraph(inputs, outputs, variables, generateBackward)


StaticGraph = Graph


def _all_nodes(outputs):
    """Every node reachable backwards from ``outputs`` (cycles through NextIteration edges allowed)."""
    seen, order, stack = set(), [], list(outputs)
    while stack:
        n = stack.pop()
        if n.id in seen:
            continue
        seen.add(n.id)
        order.append(n)
        stack.extend(n.prevs)
    return order


class DynamicGraph(Graph):
    """Graph executed by a data-flow scheduler with TensorFlow-style control flow (Switch / Merge / Enter /
    Exit / NextIteration / LoopCondition, see nn/tf.py). Reference: S/nn/DynamicGraph.scala:45-144,
    S/nn/Scheduler.scala:36-294, S/nn/FrameManager.scala:31.

    Forward runs whatever the scheduler makes ready: untaken Switch branches never run, loop bodies run once
    per iteration, and Const sub-graphs run once per model lifetime. Backward (graphs without control ops
    only, like the reference) walks the executed nodes in reverse.
    """

    def __init__(self, inputs, outputs, variables=None, generateBackward=True):
        from .scheduler import Scheduler

        inputs = list(inputs) if isinstance(inputs, (list, tuple)) else [inputs]
        outputs = list(outputs) if isinstance(outputs, (list, tuple)) else [outputs]
        Container.__init__(self)
        self.inputs_nodes = inputs
        self.output_nodes = outputs
        nodes = _all_nodes(outputs + inputs)
        nodes.sort(key=lambda n: n.id)
        self.order = nodes
        mods = [n.element for n in nodes]
        if len({id(m) for m in mods}) != len(mods):
            raise ValueError("DynamicGraph: a module instance appears in more than one node")
        self.modules = mods
        self._stop_grad = set()
        self.variables = variables
        self.generateBackward = generateBackward
        from .tf import ControlOps
        self._has_control = any(isinstance(m, ControlOps) for m in mods)
        sources = [n for n in nodes if not n.prevs]
        self.scheduler = Scheduler(sources, outputs)

    def updateOutput(self, input):
        outs = {}
        self._node_inputs = {}
        self._executed = []
        sch = self.scheduler
        sch.reset()
        while not sch.finished():
            n = sch.fetch()
            if n is None:
                break
            x = self._node_input(n, _LiveOutputs(n), input)
            self._node_inputs[n.id] = x
            outs[n.id] = n.element.forward(x)
            self._executed.append(n)
            sch.schedule(n)
        self._outs = outs
        if len(self.output_nodes) == 1:
            return self.output_nodes[0].element.output
        t = Table()
        for i, o in enumerate(self.output_nodes):
            t[i + 1] = o.element.output
        return t

    def _run_backward(self, input, gradOutput, acc_params, upd_input):
        if not self.generateBackward:
            return None
        if self._has_control:
            raise RuntimeError("DynamicGraph: backward through control-flow ops is not supported (reference "
                               "DynamicGraph.buildBackwardGraph)")
        saved = self.order
        seen, order = set(), []
        for n in self._executed:
            if n.id not in seen:
                seen.add(n.id)
                order.append(n)
        self.order = order
        try:
            return Graph._run_backward(self, input, gradOutput, acc_params, upd_input)
        finally:
            self.order = saved

    def __repr__(self):
        return f"DynamicGraph({len(self.order)} nodes)"


class _LiveOutputs:
    """Output lookup for DynamicGraph input assembly: each predecessor's live module output (a Const node
    that the scheduler skips on later forwards still holds its value)."""

    def __init__(self, node):
        self._by_id = {p.id: p.element for p in node.prevs}

    def __getitem__(self, nid):
        return self._by_id[nid].output


def Model(inputs, outputs):
    return Graph(inputs, outputs)


__all__ = ["Node", "Input", "Graph", "StaticGraph", "DynamicGraph", "Model", "topo_sort"]
