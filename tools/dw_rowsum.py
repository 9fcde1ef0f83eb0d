"""Split-operand weight-gradient GEMM (dW = dY^T X, ViT FFN1 shape) with and without the fused
bias-gradient row sums, operands pre-split: isolates the cost of a_rowsum.  python tools/dw_rowsum.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import mmfd  # noqa: E402,F401
from mmfd import kernels as K  # noqa: E402


def timeit(f, iters=10):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


for T, I, D in ((100864, 3072, 768), (100864, 768, 3072), (100864, 2304, 768), (65536, 768, 768)):
    dy = torch.randn(T, I, device="cuda"); x = torch.randn(T, D, device="cuda")
    dyp, xp = K.split3(dy), K.split3(x)
    g = torch.empty(I, D, device="cuda"); rs = torch.empty(I, device="cuda")
    t0 = timeit(lambda: K.gemm(dy, x, trans_a=True, trans_b=True, out=g, a_planes=dyp, b_planes=xp))
    t1 = timeit(lambda: K.gemm(dy, x, trans_a=True, trans_b=True, out=g, a_rowsum=rs, a_planes=dyp, b_planes=xp))
    f = 2.0 * T * I * D
    print(f"dW {I}x{D} K={T}: plain {t0:.3f} ms ({f / t0 / 1e9:.0f} TF)  +rowsum {t1:.3f} ms ({f / t1 / 1e9:.0f} TF)",
          flush=True)
