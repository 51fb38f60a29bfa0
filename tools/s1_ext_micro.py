"""The 1x1 data gradients with the extended epilogue in ResNet-50 b256 (residual addend under its sign mask, the
consumer-BN backward reduction over x with the sign mask): one line per problem and epilogue, us and effective TB/s
of the bytes it must move. Run once per BIGDL_CONV_S1 value to compare the streaming kernel with the tile kernels.
    python tools/s1_ext_micro.py"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bigdl_amd  # noqa: E402,F401
from bigdl_amd.ops import bn as bnops  # noqa: E402
from bigdl_amd.ops import conv as cv  # noqa: E402

CL, BF = torch.channels_last, torch.bfloat16


def timeit(fn, reps=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return statistics.median(ts)


def main():
    dev = torch.device("cuda")
    # (N, H, W, K = dy channels, C = dx channels): stage-3 conv1 (1024 -> 256) and stage-1 conv3 (64 -> 256) dgrads
    for (N, H, W, K, C) in ((256, 14, 14, 256, 1024), (256, 56, 56, 256, 64), (256, 28, 28, 128, 512),
                          (256, 56, 56, 64, 256)):
        P = N * H * W
        dy = (torch.randn(N, K, H, W, device=dev) * 0.1).to(BF).contiguous(memory_format=CL)
        w = (torch.randn(K, C, 1, 1, device=dev) * 0.05).to(BF)
        wt = cv.transpose_w(w)
        add = (torch.randn(N, C, H, W, device=dev) * 0.1).to(BF).contiguous(memory_format=CL)
        zm = torch.randint(0, 256, (P, C // 8), device=dev, dtype=torch.uint8)
        bx = torch.randn(N, C, H, W, device=dev).to(BF).contiguous(memory_format=CL)
        mean = torch.zeros(C, device=dev)
        out = torch.empty(N, C, H, W, device=dev, dtype=BF, memory_format=CL)

        def bn():
            return {"x": bx, "z": None, "zm": zm, "mean": mean, "aff": None, "red": bnops.new_stats(C, dev)}

        cases = [
            ("plain", P * (K + C) * 2, lambda: cv.conv2d_dgrad(dy, wt, (N, C, H, W), (1, 1), (0, 0), out=out)),
            ("bn", P * (K + 2 * C) * 2 + P * C // 8,
             lambda: cv.conv2d_dgrad(dy, wt, (N, C, H, W), (1, 1), (0, 0), out=out, bn=bn())),
            ("add+bn", P * (K + 3 * C) * 2 + P * C // 4,
             lambda: cv.conv2d_dgrad(dy, wt, (N, C, H, W), (1, 1), (0, 0), out=out, addend=add, addend_zm=zm,
                                     bn=bn())),
        ]
        for tag, nbytes, fn in cases:
            t = timeit(fn)
            print(f"S1={os.environ.get('BIGDL_CONV_S1', '2')} P={P} K={K} C={C} {tag:7s}: {t:7.1f} us "
                  f"{nbytes / t / 1e6:5.2f} TB/s of {nbytes / 1e6:.0f} MB", flush=True)


if __name__ == "__main__":
    main()
