"""Graph models: ``Graph(inputs, outputs)`` over module nodes.

Reference: S/nn/Graph.scala:72 (factories :476-560, stopGradient :248), StaticGraph.scala:38 (topological
forward :56-67, backward :82-103), DynamicGraph.scala, utils/DirectedGraph.scala:36 (topological sort).

Build with ``node = Layer(...).inputs(prev_node, ...)`` (or ``Layer(...)(prev)``); a node with several
predecessors receives a 1-based Table of their outputs in edge order. Execution follows a topological
order computed once; backward walks it in reverse, summing gradients at fan-out nodes.
"""
import time

import torch

from ..utils.table import Table
from .abstractnn import AbstractModule
from .activation import Identity
from .containers import Container, add_activity


class Node:
    _ids = 0

    def __init__(self, element):
        self.element = element
        self.prevs = []
        self.nexts = []
        Node._ids += 1
        self.id = Node._ids

    def add_next(self, node):
        self.nexts.append(node)
        node.prevs.append(self)
        return node

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
        if n in self.inputs_nodes:
            if len(self.inputs_nodes) == 1:
                return graph_input
            return graph_input[self.inputs_nodes.index(n) + 1]
        if len(n.prevs) == 1:
            return outs[n.prevs[0].id]
        t = Table()
        for i, p in enumerate(n.prevs):
            t[i + 1] = outs[p.id]
        return t

    def updateOutput(self, input):
        outs = {}
        self._node_inputs = {}
        for n in self.order:
            x = self._node_input(n, outs, input)
            self._node_inputs[n.id] = x
            outs[n.id] = n.element.forward(x)
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
            if acc_params and upd_input:
                gi = m.backward(x, g)
            elif upd_input:
                gi = m.updateGradInput(x, g)
            else:
                m.accGradParameters(x, g)
                gi = m.gradInput
            if m.hasName() and m.getName() in self._stop_grad:
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
                grads[p.id] = add_activity(grads.get(p.id), gi)
            else:
                for i, p in enumerate(n.prevs):
                    grads[p.id] = add_activity(grads.get(p.id), gi[i + 1] if gi is not None else None)
        return gin

    def backward(self, input, gradOutput):
        t0 = time.perf_counter_ns()
        self.gradInput = self._run_backward(input, gradOutput, True, True)
        self.backward_time += time.perf_counter_ns() - t0
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


StaticGraph = Graph


class DynamicGraph(Graph):
    """Graph whose execution order is decided at run time (control-flow ops); executes the same way here
    because the nodes run eagerly."""


def Model(inputs, outputs):
    return Graph(inputs, outputs)


__all__ = ["Node", "Input", "Graph", "StaticGraph", "DynamicGraph", "Model", "topo_sort"]
