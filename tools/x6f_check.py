"""Split-operand fp32 GEMM: error against an fp64 product (per operand layout, the fp32 MFMA's own
error beside it) and time on the encoder shapes (bs = 256 pairs). Run once per kernel:
  python tools/x6f_check.py                      # fused-plane kernel (default)
  MMFD_X6_SEGMENTED=1 python tools/x6f_check.py  # segmented kernel"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import mmfd  # noqa: E402,F401
from mmfd import kernels as K  # noqa: E402

DEV = "cuda"
kind = "segmented" if os.environ.get("MMFD_X6_SEGMENTED") else "fused"
print("kernel:", kind, flush=True)
for (M, N, Kd) in ((512, 768, 768), (1000, 520, 200), (300, 264, 1056), (256, 2304, 65536), (100864, 3072, 768)):
    for lay in ("nn", "nt", "tt"):
        ta, tb = lay[0] == "t", lay[1] == "t"
        if not K.x6_ok(M, N, Kd, ta, tb):
            continue
        g = torch.Generator().manual_seed(M + N + Kd)
        A = torch.randn((Kd, M) if ta else (M, Kd), generator=g).to(DEV)
        B = (torch.randn((Kd, N) if tb else (N, Kd), generator=g) * 0.05).to(DEV)
        if M * N > 10_000_000:  # check a row panel only against fp64
            rows = slice(0, 512)
            Ad = (A.double().T if ta else A.double())[rows]
        else:
            rows = slice(None)
            Ad = A.double().T if ta else A.double()
        ref = Ad @ (B.double() if tb else B.double().T)
        outs = {}
        for mode in ("split", "native"):
            K.set_fp32_gemm_mode(mode)
            outs[mode] = K.gemm(A, B, trans_a=ta, trans_b=tb)[rows]
        K.set_fp32_gemm_mode("split")
        torch.cuda.synchronize()
        sc = ref.abs().max().item()
        e = {m: (o.double() - ref).abs().max().item() / sc for m, o in outs.items()}
        print(f"err M={M} N={N} K={Kd} {lay}: split {e['split']:.3e} native {e['native']:.3e} "
              f"ratio {e['split'] / e['native']:.2f}", flush=True)


def run(M, N, Kd, layout, iters=10):
    if layout == "fwd":
        A = torch.randn(M, Kd, device=DEV); B = torch.randn(N, Kd, device=DEV); out = torch.empty(M, N, device=DEV)
        ap, bp = K.split3(A), K.split3(B)
        f = lambda: K.gemm(A, B, out=out, a_planes=ap, b_planes=bp)  # noqa: E731
    elif layout == "dx":
        A = torch.randn(M, N, device=DEV); B = torch.randn(N, Kd, device=DEV); out = torch.empty(M, Kd, device=DEV)
        ap, bp = K.split3(A), K.split3(B)
        f = lambda: K.gemm(A, B, trans_b=True, out=out, a_planes=ap, b_planes=bp)  # noqa: E731
    else:
        A = torch.randn(M, N, device=DEV); B = torch.randn(M, Kd, device=DEV); out = torch.empty(N, Kd, device=DEV)
        rs = torch.empty(N, device=DEV)
        ap, bp = K.split3(A), K.split3(B)
        f = lambda: K.gemm(A, B, trans_a=True, trans_b=True, out=out, a_planes=ap, b_planes=bp, a_rowsum=rs)  # noqa: E731
    for _ in range(2):
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


tot_ms = tot_f = 0.0
for name, M in (("bert", 65536), ("vit", 100864)):
    for lname, N, Kd in (("qkv", 2304, 768), ("out", 768, 768), ("ffn1", 3072, 768), ("ffn2", 768, 3072)):
        for layout in ("fwd", "dx", "dw"):
            ms, tf = run(M, N, Kd, layout)
            tot_ms += ms * 12
            tot_f += 2.0 * M * N * Kd * 12
            print(f"{kind} {name:5s} {lname:5s} {layout:4s} M={M:6d} N={N:5d} K={Kd:5d} {ms:8.3f} ms {tf:7.1f} TF/s "
                  f"(fp32-equivalent; {tf / 419.4:.3f} of the 419.4 TF split-operand ceiling)", flush=True)
print(f"{kind}: encoder GEMMs per step (x12 layers, operands pre-split): {tot_ms:.1f} ms, "
      f"{tot_f / tot_ms / 1e9:.1f} TF/s fp32-equivalent", flush=True)
