"""Run-to-run determinism on the GPU: N runs in one process, relative weight difference of each against the first.
  opt        Optimizer.optimize() (tests/test_optimizer_graph_gpu.py _run, eager)
  opt_sync   the same with torch.cuda.synchronize() after every iteration
  step       TrainStep.step on the same batches already on the device (no Optimizer, no DeviceFeed)
Run under env settings (BIGDL_WGRAD_STREAM=0, ...) to localise a nondeterministic path."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tests.test_optimizer_graph_gpu as T  # noqa: E402


def run_step(iters=6):
    from bigdl_amd import nn
    from bigdl_amd import optim as O
    from bigdl_amd.models.resnet import DatasetType, ResNet
    from bigdl_amd.optim.train_step import TrainStep
    from bigdl_amd.utils.random_generator import RNG

    RNG.setSeed(42)
    model = ResNet(10, 20, dataSet=DatasetType.CIFAR10)
    g = torch.Generator().manual_seed(0)
    X = torch.randn(96, 3, 32, 32, generator=g).cuda()
    Y = torch.randint(1, 11, (96,), generator=g).float().cuda()
    step = TrainStep(model, nn.CrossEntropyCriterion(), O.SGD(0.05, momentum=0.9, dampening=0.0,
                                                             learningRateDecay=0.01), device=torch.device("cuda:0"))
    for i in range(iters):
        step.step(X[16 * i:16 * (i + 1)], Y[16 * i:16 * (i + 1)])
    torch.cuda.synchronize()
    return step.w[:step.total].float().cpu().clone()


def run_opt(sync):
    if sync:
        import bigdl_amd.optim.optimizer as OM
        orig = OM.Optimizer._train_iterations

        def patched(self, *a, **k):
            hook = self._iteration_hook

            def h(n):
                torch.cuda.synchronize()
                if hook is not None:
                    hook(n)
            self._iteration_hook = h
            return orig(self, *a, **k)
        OM.Optimizer._train_iterations = patched
        try:
            return T._run(False)[0]
        finally:
            OM.Optimizer._train_iterations = orig
    return T._run(False)[0]


n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
for mode in sys.argv[2:] or ["opt", "opt_sync", "step"]:
    fn = {"opt": lambda: run_opt(False), "opt_sync": lambda: run_opt(True), "step": run_step}[mode]
    ws = [fn() for _ in range(n)]
    print(os.environ.get("DIAG_TAG", ""), mode, "rel vs run 0:",
          [f"{float((w - ws[0]).norm() / ws[0].norm()):.2e}" for w in ws[1:]], flush=True)
