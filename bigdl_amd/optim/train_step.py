"""One synchronous data-parallel training iteration on one device rank.

This is the per-rank core that the reference spreads over DistriOptimizer's two Spark jobs per iteration
(S/optim/DistriOptimizer.scala:204-396): getWeights → forward/backward → putGradients → aggregate shard →
optimize shard → sendWeightPartition. On MI355X it is:

  zero grads (one memset of the flat fp32 gradient buffer)
  forward / criterion / backward through the BigDL module protocol (HIP kernels, bf16 NHWC activations)
  reduce-scatter of the flat gradients over RCCL (ZeRO-1 shard per rank)            [N > 1]
  fused optimizer kernel on this rank's fp32 master shard, writing the bf16 compute shard
  all-gather of the bf16 compute weights over RCCL                                   [N > 1]

Layer regularizers (L1/L2) are folded into the optimizer kernel as per-segment decay (identical maths:
the reference adds lambda*w inside accGradParameters before the gradient average, which equals adding it
after the average). The whole step can be captured into a HIP graph once buffers are warm.
"""
import torch

from .. import nn
from ..optim.regularizer import L1L2Regularizer
from ..parallel.allreduce_parameter import AllReduceParameter


def fold_regularizers(model, total, device):
    """Collect L2 regularizer coefficients per parameter segment of the flat buffer; disable them in the
    modules. Returns (seg_off int64, seg_wd fp32) device tensors or None when nothing is regularized."""
    offs, vals = [], []
    off = 0
    folded_any = False
    for m in model.flattened_layers():
        if m.modules_list():
            continue
        for w, g in m._params:
            t = getattr(m, w, None)
            if t is None:
                continue
            reg = m.bRegularizer if w == "bias" else m.wRegularizer
            lam = 0.0
            if reg is not None:
                if not isinstance(reg, L1L2Regularizer) or reg.l1 != 0.0:
                    return None  # unsupported for folding: keep module-level regularization
                lam = reg.l2 * (m.scaleB if w == "bias" else m.scaleW)
            offs.append(off)
            vals.append(lam)
            off += t.numel()
            folded_any = folded_any or lam != 0.0
    if not folded_any:
        return None
    for m in model.flattened_layers():
        if m.wRegularizer is not None or m.bRegularizer is not None:
            m._reg_folded = True
    # merge consecutive equal segments
    mo, mv = [], []
    for o, v in zip(offs, vals):
        if mv and mv[-1] == v:
            continue
        mo.append(o)
        mv.append(v)
    return (torch.tensor(mo, dtype=torch.int64, device=device), torch.tensor(mv, dtype=torch.float32, device=device))


class TrainStep:
    def __init__(self, model, criterion, optim_method, device=None, comm=None, compress=None, fuse=True,
                 overlap=None, bucket_elems=8 << 20):
        from ..utils.engine import Engine

        self.device = torch.device(device) if device is not None else Engine.device()
        self.model = model
        self.criterion = criterion
        self.optim = optim_method
        model.to(self.device)
        criterion.to(self.device)
        if fuse and self.device.type == "cuda":
            from ..nn.fusion import fuse_for_training

            fuse_for_training(model)
        ws, _ = model.parameters() or ([], [])
        total = sum(w.numel() for w in ws)
        self.comm = comm if comm is not None else AllReduceParameter(total, compress=compress)
        self.w, self.g = model.getParameters(pad_multiple=max(self.comm.padded // max(total, 1), 1) if False else 1)
        if self.w.numel() != self.comm.padded:
            # re-flatten into a padded buffer so every rank's shard has the same size
            pw = torch.zeros(self.comm.padded, device=self.device)
            pg = torch.zeros(self.comm.padded, device=self.device)
            pw[:total].copy_(self.w[:total])
            model._flat = None
            self.w, self.g = _reflatten(model, pw, pg)
        self.comm.init(self.w, [t for t in (model.getExtraParameter() or [])])
        self.w16 = None
        if self.device.type == "cuda":
            self.w16 = torch.empty(self.comm.padded, dtype=torch.bfloat16, device=self.device)
            self.w16.copy_(self.w)
            model.attach_bf16_shadow(self.w16)
        seg = fold_regularizers(model, total, self.device) if self.device.type == "cuda" else None
        self.w_shard = self.comm.shard_of(self.w)
        self.g_shard = self.comm.shard_of(self.g)
        if seg is not None:
            optim_method._wd_segments = seg
            optim_method._seg_base = self.comm.start
        if self.w16 is not None:
            optim_method.attach_shadow(self.comm.shard_of(self.w16))
        self.loss = None
        self._graph = None
        # ParallelOptimizer-style bucketed reduce-scatter overlapped with backward (parallel/bucketed.py)
        from ..nn.containers import Sequential

        if overlap is None:
            overlap = self.comm.world > 1 and isinstance(model, Sequential) and compress is None
        self.bucketed = None
        if overlap and self.comm.world > 1:
            from ..parallel.bucketed import BucketedGradSync

            self.bucketed = BucketedGradSync(model, self.w, self.g, self.w16, optim_method, self.comm.world,
                                             self.comm.rank, self.comm.group, bucket_elems, total)

    def zero_grad(self):
        self.g.zero_()

    def forward_backward(self, x, y):
        m, c = self.model, self.criterion
        m.training()
        out = m.forward(x)
        loss = c.forward(out, y)
        gout = c.backward(out, y)
        if self.bucketed is not None:
            self.bucketed.backward(x, gout)
        else:
            m.backward(x, gout)
        return loss

    def sync_and_update(self, loss):
        if self.bucketed is not None:
            self.bucketed.update(loss)
            return
        self.comm.reduce_scatter_gradients(self.g, out=self.g_shard)
        self.optim.optimize(lambda _: (loss, self.g_shard), self.w_shard)
        if self.comm.world > 1:
            if self.w16 is not None:
                self.comm.all_gather_weights(self.w16)
            else:
                self.comm.all_gather_weights(self.w)

    def step(self, x, y):
        arena = None
        if self.device.type == "cuda":
            from ..ops.bn import ARENA as arena

            arena.begin(self.device)
        try:
            self.zero_grad()
            loss = self.forward_backward(x, y)
            self.sync_and_update(loss)
        finally:
            if arena is not None:
                arena.end()
        self.loss = loss
        return loss


def _reflatten(model, fw, fg):
    """Rebind every parameter of ``model`` into the given (padded) flat buffers, keeping values."""
    ws, gs = model.parameters()
    views = []
    off = 0
    from ..nn.abstractnn import _dense_strides

    for w, g in zip(ws, gs):
        n = w.numel()
        st = _dense_strides(w)
        vw = fw[off:off + n].as_strided(w.shape, st)
        vg = fg[off:off + n].as_strided(w.shape, st)
        vw.copy_(w.detach())
        vg.copy_(g.detach())
        views.append((vw, vg, off, n, st))
        off += n
    model._rebind_params(views)
    model._flat = (fw, fg)
    model._flat_views = views
    model._flat_total = off
    return fw, fg
