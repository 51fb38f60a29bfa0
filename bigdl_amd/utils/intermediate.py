"""Engine-neutral intermediate representation of a model and its lowering to the CPU or GPU engine.

Reference: S/utils/intermediate/IRGraph.scala:41-220 (IRGraph with inputs / outputs, ``build``),
IRElement.scala:27-182 (IRSpatialConvolution, IRSpatialBatchNormalization, IRLinear, IRReLU, pooling, LRN,
SoftMax, Dropout, JoinTable, CAddTable, ... and IRGeneralModule for everything else), BlasToIR.scala:28-55,
IRToBlas.scala, IRToDnn.scala:71-554 (lowering + fusion), IRConverter.scala:30-114, ConversionUtils.scala:31-95
(``convert(model)`` / ``getInt8ModelIfNeeded``), and the container-to-graph flattening of
Sequential.toGraph / DynamicContainer.toGraph.

* ``BlasToIR.convert(module)`` flattens containers (Sequential, ConcatTable, Concat, Graph) into an IRGraph whose
  nodes hold one IRElement per leaf layer: op name, the recorded constructor arguments, and the layer's
  parameters and buffers. Layers that are not in the op set become ``IRGeneralModule`` elements that carry the
  module itself, like the reference.
* ``IRToBlas`` rebuilds fresh layers from the elements (the fp32 CPU engine).
* ``IRToDnn`` rebuilds them for the GPU engine (``device``) and, for inference, runs the compile-time fusion
  passes of the MKL-DNN engine (S/nn/mkldnn/Fusion.scala:60-217): BatchNorm folded into the preceding
  convolution's weights and bias, and ReLU fused into the conv / BN epilogue.
* ``ConversionUtils.convert(model, engine)`` is the user entry point (``engine`` in {"blas", "dnn"}).
"""
import torch

from ..nn.abstractnn import module_class, module_key

IR_OPS = {"SpatialConvolution", "SpatialDilatedConvolution", "SpatialShareConvolution", "SpatialBatchNormalization",
          "BatchNormalization", "Linear", "ReLU", "SpatialMaxPooling", "SpatialAveragePooling", "SpatialCrossMapLRN",
          "SoftMax", "LogSoftMax", "Dropout", "Identity", "JoinTable", "CAddTable", "SelectTable", "Reshape",
          "View", "InferReshape", "LSTM", "GRU", "Recurrent", "TimeDistributed", "LookupTable", "Tanh", "Sigmoid"}


class IRElement:
    """One layer: op name, constructor arguments, weights (parameters + buffers) and name."""

    def __init__(self, op, args=(), kwargs=None, weights=None, name=None, module=None, attrs=None, source=None):
        self.op = op
        self.source = source if source is not None else module   # the layer this element was taken from
        self.attrs = dict(attrs or {})   # simple state set after construction (e.g. pooling .ceil())
        self.args = tuple(args)
        self.kwargs = dict(kwargs or {})
        self.weights = dict(weights or {})
        self.name = name
        self.module = module          # IRGeneralModule: the original layer

    @property
    def general(self):
        return self.module is not None

    def __repr__(self):
        return f"IR{'GeneralModule' if self.general else ''}[{self.op}]({self.name})"


class IRNode:
    _ids = 0

    def __init__(self, element):
        self.element = element
        self.prevs = []
        IRNode._ids += 1
        self.id = IRNode._ids

    def __repr__(self):
        return f"IRNode({self.element!r})"


class IRGraph:
    def __init__(self, inputs, outputs):
        self.inputs = list(inputs)
        self.outputs = list(outputs)

    def nodes(self):
        seen, order = set(), []

        def visit(n):
            if n.id in seen:
                return
            seen.add(n.id)
            for p in n.prevs:
                visit(p)
            order.append(n)

        for o in self.outputs:
            visit(o)
        for i in self.inputs:
            if i.id not in seen:
                order.insert(0, i)
                seen.add(i.id)
        return order

    def build(self, engine="blas", device=None, train=False, share=False):
        return IRConverter(self).toGraph(engine, device, train, share)

    def __repr__(self):
        return f"IRGraph({len(self.nodes())} nodes)"


# ---------------------------------------------------------------------------------------------- BlasToIR
def _weights_of(m):
    w = {}
    for wn, _ in m._params:
        t = getattr(m, wn, None)
        if isinstance(t, torch.Tensor):
            w[wn] = t.detach().clone().cpu()
    for b in m._buffers:
        t = getattr(m, b, None)
        if isinstance(t, torch.Tensor):
            w[b] = t.detach().clone().cpu()
    return w


class BlasToIR:
    @staticmethod
    def element(m):
        op = type(m).__name__
        args, kw = getattr(m, "_init_args", ((), {}))
        name = m.getName() if m.hasName() else None
        if op in IR_OPS and module_key(type(m)) == op:
            from .serializer import _SKIP_ATTRS, _is_simple
            attrs = {k: v for k, v in vars(m).items() if not k.startswith("_") and k not in _SKIP_ATTRS
                     and _is_simple(v)}
            return IRElement(op, args, kw, _weights_of(m), name, attrs=attrs, source=m)
        return IRElement(module_key(type(m)), args, kw, {}, name, module=m)

    @staticmethod
    def convert(model):
        """Flatten ``model`` into an IRGraph (one input node)."""
        inp = IRNode(IRElement("Input", name="input"))
        out = BlasToIR._lower(model, inp)
        outs = out if isinstance(out, list) else [out]
        return IRGraph([inp], outs)

    @staticmethod
    def _node(m, prevs):
        n = IRNode(BlasToIR.element(m))
        n.prevs = list(prevs)
        return n

    @staticmethod
    def _lower(m, x):
        from ..nn.containers import Concat, ConcatTable, Sequential
        from ..nn.graph import Graph
        from ..nn.table_ops import JoinTable, SelectTable

        xs = x if isinstance(x, list) else [x]
        if isinstance(m, Sequential) and type(m) is Sequential:
            for c in m.modules:
                x = BlasToIR._lower(c, x)
            return x
        if isinstance(m, ConcatTable) and type(m) is ConcatTable:
            return [BlasToIR._single(BlasToIR._lower(c, x)) for c in m.modules]
        if isinstance(m, Concat) and type(m) is Concat:
            branches = [BlasToIR._single(BlasToIR._lower(c, x)) for c in m.modules]
            return BlasToIR._node(JoinTable(m.dimension, 0), branches)
        if isinstance(m, SelectTable) and isinstance(x, list) and m.index > 0:
            return x[m.index - 1]
        if isinstance(m, Graph) and type(m) is Graph:
            mapping = {}
            for n in m.order:
                if n in m.inputs_nodes and not n.prevs:
                    k = m.inputs_nodes.index(n)
                    mapping[n.id] = xs[k] if len(m.inputs_nodes) > 1 else BlasToIR._single(x)
                    continue
                prevs = [mapping[p.id] if k is None else _select(mapping[p.id], k)
                         for p, k in zip(n.prevs, n.prev_index)]
                mapping[n.id] = BlasToIR._node(n.element, prevs)
            outs = [mapping[o.id] for o in m.output_nodes]
            return outs[0] if len(outs) == 1 else outs
        return BlasToIR._node(m, xs)

    @staticmethod
    def _single(x):
        if isinstance(x, list):        # a table-producing branch stays a list of nodes
            n = IRNode(IRElement("__table__"))
            n.prevs = list(x)
            return n
        return x


def _select(node, k):
    from ..nn.table_ops import SelectTable
    n = IRNode(BlasToIR.element(SelectTable(k)))
    n.prevs = [node]
    return n


# ---------------------------------------------------------------------------------------------- IRToBlas / IRToDnn
class IRToBlas:
    @staticmethod
    def module(e, share=False):
        """A layer for the element: the source layer itself when ``share`` (toGraph), else a rebuilt copy."""
        if e.general or (share and e.source is not None):
            return e.source
        if e.op in ("Recurrent", "BiRecurrent") and e.source is not None:
            # the cell is added after construction (Recurrent.add), not a constructor argument: copy the layer
            import copy

            m = copy.deepcopy(e.source)
            if e.name:
                m.setName(e.name)
            return m
        m = module_class(e.op)(*e.args, **e.kwargs)
        for k, v in e.attrs.items():
            if k not in ("fuse_relu", "passthrough", "emit_stats", "train"):
                setattr(m, k, v)
        with torch.no_grad():
            for k, t in e.weights.items():
                cur = getattr(m, k, None)
                if isinstance(cur, torch.Tensor) and cur.shape == t.shape:
                    cur.copy_(t)
                else:
                    setattr(m, k, t.clone())
        if e.name:
            m.setName(e.name)
        return m


def _fold_bn_into_conv(conv_e, bn_e):
    """Fold inference BatchNorm into the preceding convolution (mkldnn/Fusion.scala:173-217)."""
    w = conv_e.weights["weight"]
    b = conv_e.weights.get("bias")
    mean, var = bn_e.weights["runningMean"], bn_e.weights["runningVar"]
    eps = bn_e.kwargs.get("eps", bn_e.args[1] if len(bn_e.args) > 1 else 1e-5)
    gamma = bn_e.weights.get("weight", torch.ones_like(mean))
    beta = bn_e.weights.get("bias", torch.zeros_like(mean))
    scale = gamma / torch.sqrt(var + eps)
    out_ch = w.shape[0]
    new = IRElement(conv_e.op, conv_e.args, dict(conv_e.kwargs), dict(conv_e.weights), conv_e.name,
                    attrs=conv_e.attrs)
    new.weights["weight"] = w * scale.view((out_ch,) + (1,) * (w.dim() - 1))
    new.weights["bias"] = (b if b is not None else torch.zeros(out_ch)) * scale + beta - mean * scale
    if len(new.args) > 16:                       # withBias passed positionally
        new.args = new.args[:16] + (True,) + new.args[17:]
    else:
        new.kwargs["withBias"] = True
    return new


def _channel_affine(e, nout):
    """(scale, shift) per output channel of a Caffe-style Scale / CMul / CAdd element with a [1, C, 1, 1] (or [C])
    parameter, or None when the element is not a per-channel affine map over ``nout`` channels."""
    m = e.module if e.general else e.source
    if m is None:
        return None
    w = getattr(m, "weight", None) if e.op in ("Scale", "CMul") else None
    b = getattr(m, "bias", None) if e.op in ("Scale", "CAdd") else None
    out = []
    for t in (w, b):
        if t is None:
            out.append(None)
            continue
        t = t.detach().float().cpu()
        shape = [d for d in t.shape]
        if t.numel() != nout or (len(shape) == 4 and (shape[0] != 1 or shape[2] != 1 or shape[3] != 1)) \
                or len(shape) not in (1, 4):
            return None
        out.append(t.reshape(nout))
    if out[0] is None and out[1] is None:
        return None
    return (out[0] if out[0] is not None else torch.ones(nout)), (out[1] if out[1] is not None else torch.zeros(nout))


def _fold_affine_into_conv(conv_e, scale, shift):
    """conv -> per-channel affine (Caffe Scale after BatchNorm): W' = W * s, b' = b * s + t."""
    w = conv_e.weights["weight"]
    out_ch = w.shape[0]
    b = conv_e.weights.get("bias")
    new = IRElement(conv_e.op, conv_e.args, dict(conv_e.kwargs), dict(conv_e.weights), conv_e.name,
                    attrs=conv_e.attrs)
    new.weights["weight"] = w * scale.view((out_ch,) + (1,) * (w.dim() - 1))
    new.weights["bias"] = (b if b is not None else torch.zeros(out_ch)) * scale + shift
    if len(new.args) > 16:
        new.args = new.args[:16] + (True,) + new.args[17:]
    else:
        new.kwargs["withBias"] = True
    return new


class IRToDnn:
    """GPU-engine lowering with the inference fusion passes."""

    CONV = ("SpatialConvolution", "SpatialShareConvolution", "SpatialDilatedConvolution")
    AFFINE = ("Scale", "CMul", "CAdd")

    @staticmethod
    def _nexts(graph):
        nodes = graph.nodes()
        nexts = {n.id: [] for n in nodes}
        for n in nodes:
            for p in n.prevs:
                nexts[p.id].append(n)
        return nodes, nexts

    @staticmethod
    def _replace(graph, nodes, replaced):
        for n in nodes:
            n.prevs = [replaced.get(p.id, p) for p in n.prevs]
        graph.outputs = [replaced.get(o.id, o) for o in graph.outputs]

    @staticmethod
    def fuse(graph):
        """conv -> BN folding, then conv -> per-channel affine (Caffe BatchNorm + Scale pairs) folding, on a copy of
        the IR (inference only). ReLU / residual / concat fusion runs on the built graph
        (nn.fusion.fuse_graph_for_inference)."""
        nodes, nexts = IRToDnn._nexts(graph)
        replaced = {}
        for n in nodes:
            e = n.element
            if e.op in ("SpatialBatchNormalization",) and len(n.prevs) == 1:
                p = n.prevs[0]
                pe = p.element
                if (pe.op in IRToDnn.CONV and not pe.general and len(nexts[p.id]) == 1
                        and "runningMean" in e.weights):
                    p.element = _fold_bn_into_conv(pe, e)
                    replaced[n.id] = p
        IRToDnn._replace(graph, nodes, replaced)
        nodes, nexts = IRToDnn._nexts(graph)
        replaced = {}
        for n in nodes:      # chains conv -> Scale -> CAdd fold one after the other (nodes are in topo order)
            e = n.element
            if e.op in IRToDnn.AFFINE and len(n.prevs) == 1:
                p = replaced.get(n.prevs[0].id, n.prevs[0])
                pe = p.element
                if pe.op in IRToDnn.CONV and not pe.general and len(nexts[n.prevs[0].id]) == 1:
                    aff = _channel_affine(e, pe.weights["weight"].shape[0])
                    if aff is not None:
                        p.element = _fold_affine_into_conv(pe, *aff)
                        replaced[n.id] = p
        IRToDnn._replace(graph, nodes, replaced)
        IRToDnn._merge_lstm_stacks(graph)
        return graph

    @staticmethod
    def _plain_lstm(e):
        """The LSTM cell of a Recurrent element when it is the primitive's vanilla LSTM (no dropout, default
        activations, no batch-norm pre-topology, no masking), else None."""
        from ..nn.recurrent import LSTM, Recurrent

        m = e.source
        if e.op != "Recurrent" or not isinstance(m, Recurrent) or type(m.cell) is not LSTM:
            return None
        c = m.cell
        if m.bn is not None or m.maskZero or not c._fused_ok() or c.preTopology is None:
            return None
        return c

    @staticmethod
    def _merge_lstm_stacks(graph):
        """Chains of two or more plain Recurrent(LSTM(H, H)) layers, each the only consumer of the previous, become
        ONE nn.mkldnn.RNN(VanillaLstm, H, H, layers = L) element (the reference primitive's `layers`,
        S/nn/mkldnn/RNN.scala:87-92: stacked layers need inputSize == hiddenSize), with the weights moved into its
        ldigo layout and gate order."""
        from ..nn.mkldnn import _ORDER, AlgKind

        nodes, nexts = IRToDnn._nexts(graph)
        replaced, taken = {}, set()
        order = list(_ORDER[AlgKind.VanillaLstm])
        for n in nodes:
            c = IRToDnn._plain_lstm(n.element)
            if n.id in taken or c is None or c.inputSize != c.hiddenSize:
                continue
            H = c.hiddenSize
            chain = [n]
            while True:
                nx = nexts[chain[-1].id]
                if len(nx) != 1 or len(nx[0].prevs) != 1:
                    break
                c2 = IRToDnn._plain_lstm(nx[0].element)
                if c2 is None or c2.inputSize != H or c2.hiddenSize != H:
                    break
                chain.append(nx[0])
            if len(chain) < 2:
                continue
            L = len(chain)
            w = torch.empty(L, 1, H, 4, H)
            wi = torch.empty(L, 1, H, 4, H)
            b = torch.zeros(L, 1, 4, H)
            with torch.no_grad():
                for l, node in enumerate(chain):
                    cell = node.element.source.cell
                    w[l, 0] = cell.preTopology.weight.detach().float().cpu().view(4, H, H)[order].permute(2, 0, 1)
                    wi[l, 0] = cell.h2g.weight.detach().float().cpu().view(4, H, H)[order].permute(2, 0, 1)
                    if cell.preTopology.bias is not None:
                        b[l, 0] = cell.preTopology.bias.detach().float().cpu().view(4, H)[order]
            e = IRElement("nn.mkldnn.RNN", ("vanilla_lstm", H, H, "eltwise_tanh", "unidirectional_left2right", L),
                          {"inputFormat": "ntc"}, {"weight": w, "bias": b, "weight_i": wi}, chain[0].element.name)
            merged = IRNode(e)
            merged.prevs = list(chain[0].prevs)
            replaced[chain[-1].id] = merged
            taken.update(x.id for x in chain)
        IRToDnn._replace(graph, nodes, replaced)

    @staticmethod
    def relu_plan(g):
        """Inference fusion of a built nn.Graph for the GPU engine (ReLU into producer epilogues, residual adds and
        concats in place): see nn.fusion.fuse_graph_for_inference."""
        from ..nn.fusion import fuse_graph_for_inference

        return fuse_graph_for_inference(g)


class IRConverter:
    def __init__(self, graph):
        self.graph = graph

    def toGraph(self, engine="blas", device=None, train=False, share=False):
        from ..nn.graph import Graph, Input, Node

        ir = self.graph
        if engine == "dnn" and not train:
            ir = IRToDnn.fuse(_copy_ir(ir))
        built = {}
        inputs = []
        for n in ir.nodes():
            e = n.element
            if e.op == "Input":
                node = Input(e.name)
                inputs.append(node)
            elif e.op == "__table__":
                built[n.id] = [built[p.id] for p in n.prevs]
                continue
            else:
                node = Node(IRToBlas.module(e, share and engine == "blas"))
                for p in n.prevs:
                    src = built[p.id]
                    for s in (src if isinstance(src, list) else [src]):
                        s.add_next(node)
            built[n.id] = node
        outs = []
        for o in ir.outputs:
            b = built[o.id]
            outs.extend(b if isinstance(b, list) else [b])
        g = Graph(inputs, outs)
        if engine == "dnn":
            dev = torch.device(device) if device is not None else torch.device("cuda")
            g = g.to(dev)
            if not train:
                g.evaluate()
                IRToDnn.relu_plan(g)
        elif not train and not share:
            g.evaluate()
        return g


def _copy_ir(g):
    m = {}
    for n in g.nodes():
        c = IRNode(IRElement(n.element.op, n.element.args, n.element.kwargs, dict(n.element.weights),
                             n.element.name, n.element.module, n.element.attrs, n.element.source))
        c.prevs = [m[p.id] for p in n.prevs]
        m[n.id] = c
    return IRGraph([m[i.id] for i in g.inputs], [m[o.id] for o in g.outputs])


class ConversionUtils:
    @staticmethod
    def convert(model, engine="blas", device=None, train=None):
        """Model -> IR -> engine graph (ConversionUtils.convert). ``train`` defaults to the model's mode."""
        train = model.train if train is None else train
        return BlasToIR.convert(model).build(engine, device, train)

    @staticmethod
    def getInt8ModelIfNeeded(model, quantize):
        if not quantize:
            return model
        from ..quantized.quantizer import quantize

        return quantize(model)


__all__ = ["IRElement", "IRNode", "IRGraph", "BlasToIR", "IRToBlas", "IRToDnn", "IRConverter", "ConversionUtils",
           "IR_OPS"]
