"""GEMM throughput on the hot-path shapes (BERT M=65536, ViT M=100864 tokens at bs=256 pairs).
python tools/gemm_bench.py [--dtype bf16|fp32] [--fp32-mode split|native] [--iters N]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import mmfd  # noqa: E402
from mmfd import kernels as K  # noqa: E402


def run(M, N, Kd, layout, dt, iters, lib=False):
    dev = "cuda"
    if layout == "fwd":      # y[M,N] = x[M,K] W[N,K]^T
        A = torch.randn(M, Kd, device=dev).to(dt); B = torch.randn(N, Kd, device=dev).to(dt)
        f = lambda: K.gemm(A, B, out=out)  # noqa: E731
        out = torch.empty(M, N, device=dev, dtype=dt)
    elif layout == "dx":     # dx[M,K] = dy[M,N] W[N,K]   -> (M, Kd) output, reduction N
        A = torch.randn(M, N, device=dev).to(dt); B = torch.randn(N, Kd, device=dev).to(dt)
        out = torch.empty(M, Kd, device=dev, dtype=dt)
        f = lambda: K.gemm(A, B, trans_b=True, out=out)  # noqa: E731
    else:                    # dW[N,K] = dy[M,N]^T x[M,K]
        A = torch.randn(M, N, device=dev).to(dt); B = torch.randn(M, Kd, device=dev).to(dt)
        out = torch.empty(N, Kd, device=dev, dtype=torch.float32)
        f = lambda: K.gemm(A, B, trans_a=True, trans_b=True, out=out)  # noqa: E731
    if lib:  # the same product through torch.matmul (hipBLASLt), for comparison only
        if layout == "fwd":
            f = lambda: torch.matmul(A, B.t(), out=out)  # noqa: E731
        elif layout == "dx":
            f = lambda: torch.matmul(A, B, out=out)  # noqa: E731
        else:
            out = out.to(dt)
            f = lambda: torch.matmul(A.t(), B, out=out)  # noqa: E731
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        f()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    return ms, 2.0 * M * N * Kd / (ms * 1e-3) / 1e12


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--lib", action="store_true", help="also time torch.matmul (hipBLASLt)")
    ap.add_argument("--fp32-mode", default="split", choices=["split", "native"])
    a = ap.parse_args()
    K.set_fp32_gemm_mode(a.fp32_mode)
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    tot_ms = tot_f = 0.0
    for name, M in (("bert", 65536), ("vit", 100864)):
        for lname, N, Kd in (("qkv", 2304, 768), ("out", 768, 768), ("ffn1", 3072, 768), ("ffn2", 768, 3072)):
            for layout in ("fwd", "dx", "dw"):
                ms, tf = run(M, N, Kd, layout, dt, a.iters)
                lms, ltf = run(M, N, Kd, layout, dt, a.iters, lib=True) if a.lib else (0.0, 0.0)
                tot_ms += ms * 12
                tot_f += 2.0 * M * N * Kd * 12
                print(f"{name:5s} {lname:5s} {layout:4s} M={M:6d} N={N:5d} K={Kd:5d}  {ms:8.3f} ms  {tf:7.1f} TF/s"
                      + (f"   hipBLASLt {lms:8.3f} ms {ltf:7.1f} TF/s" if a.lib else ""), flush=True)
    print(f"encoder GEMMs per step (x12 layers): {tot_ms:.1f} ms, {tot_f / tot_ms / 1e9:.1f} TF/s")
