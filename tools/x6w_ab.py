"""Split-operand fp32 GEMM: the four-wave AGPR kernel (gemm256_x6w_kernel) against the eight-wave
ping-pong kernel (gemm256_x6f_kernel), interleaved in one process on the encoder GEMM shapes of the
bs = 256 step (pre-split operands, the bench's epilogues): bitwise equality of C (and of the fused
bias-gradient row sums) and time per launch.
  python tools/x6w_ab.py [reps]"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import mmfd  # noqa: E402,F401
from mmfd import kernels as K  # noqa: E402

DEV = "cuda"
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
lib = K.lib()
lib.mmfd_debug_set_x6w.argtypes = [ctypes.c_int]
lib.mmfd_debug_set_x6w.restype = ctypes.c_int
K.set_fp32_gemm_mode("split")
g = torch.Generator(DEV).manual_seed(0)

SHAPES = [  # (name, M, N, K, kind, act): kind fwd = X W^T, dx = dY W, dw = dY^T X (+ row sums)
    ("bert qkv fwd", 65536, 2304, 768, "fwd", None), ("bert ffn1 fwd", 65536, 3072, 768, "fwd", "gelu"),
    ("bert ffn2 fwd", 65536, 768, 3072, "fwd", "res"), ("vit ffn1 fwd", 100864, 3072, 768, "fwd", "gelu"),
    ("vit ffn2 fwd", 100864, 768, 3072, "fwd", "res"), ("vit ffn1 dx", 100864, 768, 3072, "dx", None),
    ("vit ffn2 dx", 100864, 3072, 768, "dx", "gelu_bwd"), ("vit ffn1 dw", 3072, 768, 100864, "dw", None),
    ("vit qkv dw", 2304, 768, 100864, "dw", None), ("bert ffn2 dw", 768, 3072, 65536, "dw", None),
]


def make(M, N, Kd, kind, act):
    if kind == "fwd":
        A = torch.randn(M, Kd, device=DEV, generator=g); B = torch.randn(N, Kd, device=DEV, generator=g) * 0.05
        kw = {}
    elif kind == "dx":
        A = torch.randn(M, Kd, device=DEV, generator=g); B = torch.randn(Kd, N, device=DEV, generator=g) * 0.05
        kw = dict(trans_b=True)
    else:
        A = torch.randn(Kd, M, device=DEV, generator=g); B = torch.randn(Kd, N, device=DEV, generator=g) * 0.05
        kw = dict(trans_a=True, trans_b=True)
    ap = K.split3(A)
    bp = K.split3(B)
    out = torch.empty(M, N, device=DEV)
    extra = {}
    if act == "gelu":
        extra = dict(bias=torch.randn(N, device=DEV, generator=g), act=K.ACT_GELU, aux=torch.empty(M, N, device=DEV))
    elif act == "res":
        extra = dict(bias=torch.randn(N, device=DEV, generator=g), residual=torch.randn(M, N, device=DEV, generator=g))
    elif act == "gelu_bwd":
        extra = dict(act=K.ACT_GELU_BWD, aux=torch.randn(M, N, device=DEV, generator=g))
    if kind == "dw":
        extra["a_rowsum"] = torch.empty(M, device=DEV)

    def f():
        return K.gemm(A, B, out=out, a_planes=ap, b_planes=bp, **kw, **extra)
    return f, out, extra


def timed(f, n):
    f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / n


tot = {0: 0.0, 1: 0.0}
for name, M, N, Kd, kind, act in SHAPES:
    f, out, extra = make(M, N, Kd, kind, act)
    res = {}
    for w in (0, 1):
        lib.mmfd_debug_set_x6w(w)
        f()
        torch.cuda.synchronize()
        res[w] = (out.clone(), extra["a_rowsum"].clone() if "a_rowsum" in extra else None)
    same = torch.equal(res[0][0], res[1][0]) and (res[0][1] is None or torch.equal(res[0][1], res[1][1]))
    ts = {0: [], 1: []}
    for _ in range(reps):
        for w in (0, 1):
            lib.mmfd_debug_set_x6w(w)
            ts[w].append(timed(f, 5))
    fl = 2.0 * M * N * Kd
    b = {w: min(v) for w, v in ts.items()}
    for w in (0, 1):
        tot[w] += b[w]
    print(f"{name:14s} M={M} N={N} K={Kd}: x6f {b[0]:8.1f} us ({fl / b[0] / 1e6:6.1f} TF) | x6w {b[1]:8.1f} us "
          f"({fl / b[1] / 1e6:6.1f} TF) | {b[0] / b[1]:.3f}x | bitwise equal: {same}", flush=True)
    del f, out, extra, res
    torch.cuda.empty_cache()
print(f"sum of best launches: x6f {tot[0]:.1f} us, x6w {tot[1]:.1f} us ({tot[0] / tot[1]:.3f}x)")
lib.mmfd_debug_set_x6w(0)
