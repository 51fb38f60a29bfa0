"""Which reference cycles keep GPU tensors alive across training steps (GPU diagnostic).

    python tools/diag_cycles.py [--batch 64] [--image 224] [--steps 4]

Runs TrainStep on ResNet-50 with the cyclic collector disabled, then collects with DEBUG_SAVEALL and reports the
object types in the unreachable cycles, the CUDA bytes they hold, and for the largest held tensors the chain of
referrer types back into the cycle. A training step should leave no cycle holding device memory: anything here is
memory that only a GC pass returns (the caching allocator then grows between passes).
"""
import argparse
import gc
import os
import sys
from collections import Counter

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bigdl_amd  # noqa: F401,E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--image", type=int, default=224)
    ap.add_argument("--steps", type=int, default=4)
    a = ap.parse_args()
    from bigdl_amd import nn
    from bigdl_amd.models.resnet import DatasetType, ResNet
    from bigdl_amd.optim.sgd import SGD
    from bigdl_amd.optim.train_step import TrainStep
    from bigdl_amd.utils.engine import Engine

    Engine.init(master="local[1]", dist=False)
    dev = torch.device("cuda", 0)
    model = ResNet(1000, 50, dataSet=DatasetType.ImageNet)
    step = TrainStep(model, nn.CrossEntropyCriterion(), SGD(learningRate=0.1, momentum=0.9), device=dev)
    x = torch.randn(a.batch, 3, a.image, a.image, device=dev)
    y = torch.randint(1, 1001, (a.batch,), device=dev).float()
    for _ in range(2):
        step.step(x, y)
    torch.cuda.synchronize()
    gc.collect()
    gc.disable()
    base = torch.cuda.memory_allocated(dev)
    for _ in range(a.steps):
        step.step(x, y)
    torch.cuda.synchronize()
    grown = torch.cuda.memory_allocated(dev) - base
    gc.set_debug(gc.DEBUG_SAVEALL)
    n = gc.collect()
    garbage = list(gc.garbage)
    gc.set_debug(0)
    types = Counter(type(o).__name__ for o in garbage)
    tens = [o for o in garbage if torch.is_tensor(o) and o.is_cuda]
    held = sum(t.untyped_storage().nbytes() for t in tens)
    print(f"allocated growth over {a.steps} steps with GC off: {grown / 2**20:.1f} MiB; unreachable objects {n}; "
          f"CUDA tensors among them {len(tens)} holding {held / 2**20:.1f} MiB")
    print("object types in cycles:", types.most_common(25))
    ids = {id(o) for o in garbage}
    for t in sorted(tens, key=lambda t: -t.untyped_storage().nbytes())[:6]:
        chain, cur = [], t
        for _ in range(6):
            refs = [r for r in gc.get_referrers(cur) if id(r) in ids and r is not garbage]
            if not refs:
                break
            cur = refs[0]
            desc = type(cur).__name__
            if isinstance(cur, dict):
                keys = [k for k, v in cur.items() if v is t or v is chain[-1:] and False][:3]
                desc += f"(keys~{list(cur.keys())[:6]})"
            elif hasattr(cur, "__qualname__"):
                desc += f"({cur.__qualname__})"
            chain.append(desc)
        print(f"tensor {tuple(t.shape)} {t.dtype} {t.untyped_storage().nbytes() / 2**20:.1f} MiB <- " + " <- ".join(chain))
    frames = [o for o in garbage if type(o).__name__ == "frame"]
    for f in frames[:8]:
        print("frame:", f.f_code.co_filename, f.f_code.co_name, f.f_lineno)
    funcs = [o for o in garbage if type(o).__name__ == "function"]
    for f in funcs[:12]:
        print("function:", f.__qualname__, getattr(f.__code__, "co_filename", ""))
    cells = [o for o in garbage if type(o).__name__ == "cell"]
    print("cells:", len(cells))
    Engine.shutdown()


if __name__ == "__main__":
    main()
