"""Which framework lines still launch aten / runtime-memset work in the LSTM LM step (GPU): torch.profiler over two
training steps of tools/bench_lstm.py's model, aten ops that launch GPU work listed with their Python call sites.

    python tools/diag_lm_aten.py [--batch 128]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--seq", type=int, default=64)
    a = ap.parse_args()
    from bigdl_amd import nn
    from bigdl_amd.models.rnn import PTBModel
    from bigdl_amd.optim.sgd import SGD
    from bigdl_amd.optim.train_step import TrainStep

    dev = torch.device("cuda")
    model = PTBModel.lstm(10000, 1024, 10000, 2)
    crit = nn.TimeDistributedCriterion(nn.CrossEntropyCriterion(), True)
    step = TrainStep(model, crit, SGD(learningRate=1.0), device=dev)
    x = torch.randint(1, 10001, (a.batch, a.seq), device=dev).float()
    y = torch.randint(1, 10001, (a.batch, a.seq), device=dev).float()
    for _ in range(3):
        step.step(x, y)
    torch.cuda.synchronize()
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    with torch.profiler.profile(activities=acts, with_stack=True, record_shapes=False) as prof:
        for _ in range(2):
            step.step(x, y)
        torch.cuda.synchronize()
    seen = {}
    for ev in prof.events():
        name = ev.name
        if not name.startswith("aten::") or name in ("aten::empty", "aten::empty_strided", "aten::view", "aten::as_strided",
                                                     "aten::select", "aten::slice", "aten::reshape", "aten::detach",
                                                     "aten::alias", "aten::t", "aten::transpose", "aten::permute",
                                                     "aten::unsqueeze", "aten::squeeze", "aten::narrow", "aten::expand",
                                                     "aten::_reshape_alias", "aten::result_type", "aten::item",
                                                     "aten::_local_scalar_dense", "aten::lift_fresh", "aten::resolve_conj",
                                                     "aten::resolve_neg", "aten::is_nonzero", "aten::contiguous",
                                                     "aten::unbind", "aten::split", "aten::chunk", "aten::set_",
                                                     "aten::record_stream", "aten::_unsafe_view", "aten::empty_like",
                                                     "aten::new_empty", "aten::new_empty_strided", "aten::flatten",
                                                     "aten::numpy_T", "aten::dim", "aten::size", "aten::stride"):
            continue
        if ev.device_type != torch.autograd.DeviceType.CPU:
            continue
        stack = [s for s in (ev.stack or []) if "bigdl_amd" in s or "tools/" in s][:4]
        key = (name, tuple(stack))
        seen[key] = seen.get(key, 0) + 1
    for (name, stack), n in sorted(seen.items(), key=lambda kv: -kv[1]):
        print(f"{n // 2:4d}/step  {name}")
        for s in stack:
            print(f"            {s}")
    # GPU side: every kernel / memset / copy by name; an aten op that launched device work, with its Python frames
    gpu = {}
    for ev in prof.events():
        if ev.device_type != torch.autograd.DeviceType.CPU:
            key = ev.name[:90]
            gpu[key] = gpu.get(key, 0) + 1
    print("GPU work per step:")
    for name, n in sorted(gpu.items(), key=lambda kv: -kv[1]):
        print(f"{n / 2:6.1f}/step  {name}")
    print("aten ops that launched device work:")
    seen2 = {}
    for ev in prof.events():
        if ev.device_type != torch.autograd.DeviceType.CPU or not ev.name.startswith("aten::"):
            continue
        ks = [k.name[:60] for k in getattr(ev, "kernels", [])]
        if not ks:
            continue
        stack = tuple(s for s in (ev.stack or []) if "site-packages" not in s and "dist-packages" not in s)[:5]
        key = (ev.name, tuple(sorted(set(ks))), stack)
        seen2[key] = seen2.get(key, 0) + 1
    for (name, ks, stack), n in sorted(seen2.items(), key=lambda kv: -kv[1]):
        print(f"{n / 2:6.1f}/step  {name}: {', '.join(ks)}")
        for s in stack:
            print(f"            {s}")

if __name__ == "__main__":
    main()
