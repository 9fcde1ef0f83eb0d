"""The same products on three operand distributions (zeros, torch.randn, uniform [-2, 2)): the
four-wave kernel, gemm256_kernel and hipBLASLt (torch.matmul, no bias). MFMA power - and the clock
the chip holds - depends on the operand bits."""
import os
import sys

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

import mmfd.kernels as K  # noqa: E402

dev = torch.device("cuda", 0)


def t(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


for name, M, N, Kd in (("bert qkv", 65536, 2304, 768), ("vit qkv", 100864, 2304, 768)):
    for dist in ("zeros", "randn", "uniform"):
        if dist == "zeros":
            A = torch.zeros(M, Kd, device=dev, dtype=torch.bfloat16); B = torch.zeros(N, Kd, device=dev, dtype=torch.bfloat16)
        elif dist == "randn":
            A = torch.randn(M, Kd, device=dev).bfloat16(); B = torch.randn(N, Kd, device=dev).bfloat16()
        else:
            A = (torch.rand(M, Kd, device=dev) * 4 - 2).bfloat16(); B = (torch.rand(N, Kd, device=dev) * 4 - 2).bfloat16()
        bias = torch.randn(N, device=dev)
        K.set_g4_mode("on")
        g4 = t(lambda: K.gemm(A, B, bias=bias))
        K.set_g4_mode("off")
        g8 = t(lambda: K.gemm(A, B, bias=bias))
        lib = t(lambda: torch.matmul(A, B.t()))
        print(f"{name:9s} {dist:8s} g4 {g4:7.1f} us  g8 {g8:7.1f} us  hipBLASLt {lib:7.1f} us", flush=True)
