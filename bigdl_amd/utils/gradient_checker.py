"""Finite-difference gradient checks (reference T/nn/GradientChecker.scala:33, checkLayer :56, checkWeight
:163). Works on the CPU engine in fp64: the module is temporarily run on double tensors where its math
allows (torch ops upcast), so the check is independent of the module's analytic backward."""
import torch

from .table import Table


def _flat_inputs(x):
    if isinstance(x, torch.Tensor):
        return [x]
    return [t for t in x.toSeq()]


class GradientChecker:
    def __init__(self, stepSize=1e-3, threshold=1e-2):
        self.stepSize = stepSize
        self.threshold = threshold

    def _loss(self, module, x, proj):
        out = module.forward(x)
        outs = _flat_inputs(out) if not isinstance(out, torch.Tensor) else [out]
        return sum((o.double() * p).sum() for o, p in zip(outs, proj))

    def checkLayer(self, module, input, epsilon=None, seed=0):
        """Compare module.backward(input, proj) against central differences of <module(x), proj>."""
        eps = epsilon or self.stepSize
        g = torch.Generator().manual_seed(seed)
        out = module.forward(input)
        outs = _flat_inputs(out) if not isinstance(out, torch.Tensor) else [out]
        proj = [torch.randn(o.shape, generator=g, dtype=torch.float64) for o in outs]
        gout = proj[0].to(outs[0].dtype) if isinstance(out, torch.Tensor) else Table(*[p.to(o.dtype) for p, o in zip(proj, outs)])
        module.zeroGradParameters()
        gin = module.backward(input, gout)
        analytic = _flat_inputs(gin) if not isinstance(gin, torch.Tensor) else [gin]
        ok = True
        worst = 0.0
        for xi, ai in zip(_flat_inputs(input), analytic):
            if not xi.is_floating_point():
                continue
            flat = xi.view(-1)
            an = ai.reshape(-1).double()
            idx = torch.randperm(flat.numel(), generator=g)[:32]
            for j in idx.tolist():
                orig = flat[j].item()
                flat[j] = orig + eps
                lp = self._loss(module, input, proj).item()
                flat[j] = orig - eps
                lm = self._loss(module, input, proj).item()
                flat[j] = orig
                num = (lp - lm) / (2 * eps)
                err = abs(num - an[j].item()) / max(1.0, abs(num), abs(an[j].item()))
                worst = max(worst, err)
                ok = ok and err < self.threshold
        module.forward(input)
        return ok, worst

    def checkWeight(self, module, input, epsilon=None, seed=0):
        eps = epsilon or self.stepSize
        g = torch.Generator().manual_seed(seed)
        out = module.forward(input)
        outs = [out] if isinstance(out, torch.Tensor) else _flat_inputs(out)
        proj = [torch.randn(o.shape, generator=g, dtype=torch.float64) for o in outs]
        gout = proj[0].to(outs[0].dtype) if isinstance(out, torch.Tensor) else Table(*[p.to(o.dtype) for p, o in zip(proj, outs)])
        module.zeroGradParameters()
        module.backward(input, gout)
        ws, gs = module.parameters()
        worst = 0.0
        for w, gw in zip(ws, gs):
            flat = w.data.view(-1) if w.is_contiguous() else None
            if flat is None:
                continue
            an = gw.reshape(-1).double()
            idx = torch.randperm(flat.numel(), generator=g)[:16]
            for j in idx.tolist():
                orig = flat[j].item()
                flat[j] = orig + eps
                lp = self._loss(module, input, proj).item()
                flat[j] = orig - eps
                lm = self._loss(module, input, proj).item()
                flat[j] = orig
                num = (lp - lm) / (2 * eps)
                err = abs(num - an[j].item()) / max(1.0, abs(num), abs(an[j].item()))
                worst = max(worst, err)
        module.forward(input)
        return worst < self.threshold, worst
