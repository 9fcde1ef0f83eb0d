"""The split-operand fp32 GEMM (x6f) at the BERT FFN1 shape (M = 65,536, N = 3,072, K = 768) under
its epilogue variants: what the GELU math, the aux store and the planes store each cost per launch.
python tools/x6f_epi_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from mmfd import kernels as K  # noqa: E402


def timed(f, it=10):
    f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e30
    for _ in range(3):
        e0.record()
        for _ in range(it):
            f()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / it * 1e3)
    return best


def main():
    M, N, Kd = 65536, 3072, 768
    g = torch.Generator(device="cuda").manual_seed(0)
    A = torch.randn(M, Kd, device="cuda", generator=g)
    W = torch.randn(N, Kd, device="cuda", generator=g) * 0.03
    b = torch.randn(N, device="cuda", generator=g)
    ap, wp = K.split3(A), K.split3(W)
    out = torch.empty(M, N, device="cuda")
    aux = torch.empty(M, N, device="cuda")
    pl = torch.empty(3, M, N, device="cuda", dtype=torch.bfloat16)
    dy = torch.randn(M, Kd, device="cuda", generator=g)
    W2 = torch.randn(Kd, N, device="cuda", generator=g) * 0.03
    dyp, w2p = K.split3(dy), K.split3(W2)
    flop = 2.0 * M * N * Kd
    cases = [
        ("bias, C", lambda: K.gemm(A, W, bias=b, out=out, a_planes=ap, b_planes=wp)),
        ("bias, planes only", lambda: K.gemm(A, W, bias=b, out=out, a_planes=ap, b_planes=wp, out_planes=pl,
                                              write_out=False)),
        ("bias+GELU, planes only", lambda: K.gemm(A, W, bias=b, act=K.ACT_GELU, out=out, a_planes=ap, b_planes=wp,
                                                   out_planes=pl, write_out=False)),
        ("bias+GELU+pre aux, planes", lambda: K.gemm(A, W, bias=b, act=K.ACT_GELU, aux=aux, out=out, a_planes=ap,
                                                      b_planes=wp, out_planes=pl, write_out=False)),
        ("bias+GELU_D aux, planes", lambda: K.gemm(A, W, bias=b, act=K.ACT_GELU_D, aux=aux, out=out, a_planes=ap,
                                                    b_planes=wp, out_planes=pl, write_out=False)),
        ("dX x aux (MUL_AUX), planes", lambda: K.gemm(dy, W2, trans_b=True, act=K.ACT_MUL_AUX, aux=aux, out=out,
                                                       a_planes=dyp, b_planes=w2p, out_planes=pl, write_out=False)),
        ("dX x gelu'(pre), planes", lambda: K.gemm(dy, W2, trans_b=True, act=K.ACT_GELU_BWD, aux=aux, out=out,
                                                    a_planes=dyp, b_planes=w2p, out_planes=pl, write_out=False)),
        ("dX plain, C", lambda: K.gemm(dy, W2, trans_b=True, out=out, a_planes=dyp, b_planes=w2p)),
    ]
    for name, f in cases:
        us = timed(f)
        print(f"RESULT {name:32s} {us:8.1f} us  {flop / us / 1e6:6.1f} TF/s  frac {flop / us / 1e6 / 419.4:.3f}", flush=True)


if __name__ == "__main__":
    main()
