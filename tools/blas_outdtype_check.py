"""Precision of torch.mm(bf16, bf16, out_dtype=float32) / torch.addmm(..., out_dtype=float32) on this ROCm build
against a float64 reference (an fp32-output GEMM should land at ~1e-6 relative, a bf16-rounded output at ~2e-3)."""
import torch


def rel(a, b):
    return ((a.double() - b).norm() / b.norm()).item()


def main():
    torch.manual_seed(0)
    for (M, N, K) in ((4096, 1024, 32768), (10000, 1032, 32768), (2048, 2048, 8192)):
        a = torch.randn(K, M, device="cuda").to(torch.bfloat16)
        b = torch.randn(K, N, device="cuda").to(torch.bfloat16)
        ref = a.double().t() @ b.double()
        c1 = torch.mm(a.t(), b, out_dtype=torch.float32)
        c2 = torch.mm(a.float().t(), b.float())
        acc = torch.zeros(M, N, device="cuda")
        torch.addmm(acc, a.t(), b, out_dtype=torch.float32, out=acc)
        print(f"M={M} N={N} K={K}: mm(out_dtype=f32) rel {rel(c1, ref):.2e} dtype {c1.dtype} | fp32 mm rel "
              f"{rel(c2, ref):.2e} | addmm(out=acc) rel {rel(acc, ref):.2e}", flush=True)


if __name__ == "__main__":
    main()
