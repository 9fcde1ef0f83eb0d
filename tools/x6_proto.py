"""Prototype: fp32 GEMM as six bf16 split products (x = h + m + l, bf16 each), emulated with the
existing bf16 256x256 kernel on K-concatenated operands. Prints time and error vs fp64 beside the
native fp32 MFMA GEMM.  python tools/x6_proto.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import mmfd  # noqa: E402,F401
from mmfd import kernels as K  # noqa: E402


def split3(x):
    h = x.to(torch.bfloat16)
    r = x - h.float()
    m = r.to(torch.bfloat16)
    l = (r - m.float()).to(torch.bfloat16)
    return h, m, l


def timeit(f, iters=10):
    for _ in range(2):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


for (M, N, Kd) in ((100864, 3072, 768), (100864, 768, 3072), (65536, 2304, 768), (16384, 3072, 768)):
    A = torch.randn(M, Kd, device="cuda")
    B = torch.randn(N, Kd, device="cuda") * 0.02
    ah, am, al = split3(A)
    bh, bm, bl = split3(B)
    A6 = torch.cat([ah, ah, am, ah, al, am], 1).contiguous()
    B6 = torch.cat([bh, bm, bh, bl, bh, bm], 1).contiguous()
    o32 = torch.empty(M, N, device="cuda")
    o6 = torch.empty(M, N, device="cuda")
    t32 = timeit(lambda: K.gemm(A, B, out=o32))
    t6 = timeit(lambda: K.gemm(A6, B6, out=o6))
    tsplit = timeit(lambda: split3(A))
    rows = slice(0, 2048)
    ref = A[rows].double() @ B.double().t()
    e32 = ((o32[rows].double() - ref).abs().max() / ref.abs().max()).item()
    e6 = ((o6[rows].double() - ref).abs().max() / ref.abs().max()).item()
    f = 2.0 * M * N * Kd
    print(f"M={M} N={N} K={Kd}: fp32 {t32:.3f} ms ({f / t32 / 1e9:.1f} TF)  x6 {t6:.3f} ms "
          f"({f / t6 / 1e9:.1f} fp32-eq TF, {6 * f / t6 / 1e9:.0f} bf16 TF)  torch-split {tsplit:.3f} ms  "
          f"err fp32 {e32:.2e} x6 {e6:.2e}", flush=True)
