import os, sys
sys.path.insert(0, os.getcwd())
import torch, mmfd
from mmfd import kernels as K
dev = "cuda"
def t(f, it=20):
    for _ in range(3): f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it): f()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3
for M, N, Kd in ((65536, 3072, 768), (65536, 2304, 768), (65536, 768, 3072), (100864, 3072, 768)):
    A = torch.randn(M, Kd, device=dev).bfloat16(); B = torch.randn(N, Kd, device=dev).bfloat16()
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    b = torch.randn(N, device=dev)
    aux = torch.empty_like(out)
    fl = 2 * M * N * Kd
    tn = t(lambda: K.gemm(A, B, out=out))
    ts = t(lambda: K.gemm(A, B, out=out, alpha=12345.0))
    tg = t(lambda: K.gemm(A, B, out=out, bias=b, act=K.ACT_GELU, aux=aux))
    res = torch.randn(M, N, device=dev).bfloat16()
    tr = t(lambda: K.gemm(A, B, out=out, bias=b, residual=res))
    tb = t(lambda: K.gemm(A, B, out=out, act=K.ACT_GELU_BWD, aux=aux))
    print(f"   bias+residual {tr:7.1f} us ({fl/tr/1e6:6.1f})   gelu_bwd(aux) {tb:7.1f} us ({fl/tb/1e6:6.1f})", flush=True)
    print(f"M={M} N={N} K={Kd}: plain {tn:7.1f} us ({fl/tn/1e6:6.1f} TF/s)  no-epilogue {ts:7.1f} us ({fl/ts/1e6:6.1f})  bias+gelu+aux {tg:7.1f} us ({fl/tg/1e6:6.1f})", flush=True)
