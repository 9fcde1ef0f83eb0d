"""Epilogue cost on the K=768 / K=3072 encoder shapes: plain store vs. no epilogue (alpha = 12345
is the 256x256 kernel's experiment switch that skips the epilogue) vs. the fused epilogues of the
step.
python tools/epi_exp.py"""
import os
import sys

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

import mmfd  # noqa: E402,F401
from mmfd import kernels as K  # noqa: E402

dev = "cuda"


def t(f, it=20):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


for M, N, Kd in ((65536, 3072, 768), (65536, 2304, 768), (65536, 768, 3072), (100864, 3072, 768)):
    A = torch.randn(M, Kd, device=dev).bfloat16()
    B = torch.randn(N, Kd, device=dev).bfloat16()
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    b = torch.randn(N, device=dev)
    aux = torch.empty_like(out)
    res = torch.randn(M, N, device=dev).bfloat16()
    fl = 2 * M * N * Kd
    fns = {"plain": lambda: K.gemm(A, B, out=out),
           "no-epilogue": lambda: K.gemm(A, B, out=out, alpha=12345.0),
           "staging-only": lambda: K.gemm(A, B, out=out, alpha=23456.0),
           "bias+gelu+aux": lambda: K.gemm(A, B, out=out, bias=b, act=K.ACT_GELU, aux=aux),
           "bias+residual": lambda: K.gemm(A, B, out=out, bias=b, residual=res),
           "gelu_bwd(aux)": lambda: K.gemm(A, B, out=out, act=K.ACT_GELU_BWD, aux=aux)}
    r = {k: 1e30 for k in fns}
    for _ in range(3):  # interleaved rounds, best of three (clock / thermal drift between variants)
        for k, f in fns.items():
            r[k] = min(r[k], t(f))
    print(f"M={M} N={N} K={Kd}: " + "  ".join(f"{k} {v:7.1f} us ({fl / v / 1e6:6.1f} TF/s)" for k, v in r.items()),
          flush=True)

