"""The 256x256 GEMM on the encoder shapes of the step (ViT M=100864 / BERT M=65536 tokens) with the
step's epilogues (GELU + saved pre-activation, GELU backward from the saved pre-activation, residual,
bias), best of 3 x 10 launches each, plus an output checksum (tools/ab.sh compares two builds).
python tools/gemm_epi_bench.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    sys.path.insert(0, ROOT)
    import torch
    import mmfd  # noqa: F401
    from mmfd import kernels as K
    dev = "cuda"

    def t(f, it=10):
        for _ in range(2):
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

    res = {}
    for M in (100864, 65536):
        for name, N, Kd, kind in (("ffn1_fwd_gelu", 3072, 768, "gelu"), ("ffn2_dx_gelubwd", 3072, 768, "gelubwd"),
                                  ("ffn2_fwd_res", 768, 3072, "res"), ("qkv_fwd", 2304, 768, "bias"),
                                  ("out_dx", 768, 768, "dx"), ("ffn1_dx", 768, 3072, "dx")):
            g = torch.Generator(device=dev).manual_seed(0)
            A = torch.randn(M, Kd, device=dev, generator=g).bfloat16()
            out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            b = torch.randn(N, device=dev, generator=g)
            if kind == "dx":
                B = torch.randn(Kd, N, device=dev, generator=g).bfloat16()
                f = lambda: K.gemm(A, B, trans_b=True, out=out)  # noqa: E731
            else:
                B = torch.randn(N, Kd, device=dev, generator=g).bfloat16()
                aux = torch.randn(M, N, device=dev, generator=g).bfloat16()
                if kind == "gelu":
                    f = lambda: K.gemm(A, B, out=out, bias=b, act=K.ACT_GELU, aux=aux)  # noqa: E731
                elif kind == "gelubwd":
                    f = lambda: K.gemm(A, B, out=out, act=K.ACT_GELU_BWD, aux=aux)  # noqa: E731
                elif kind == "res":
                    f = lambda: K.gemm(A, B, out=out, bias=b, residual=aux)  # noqa: E731
                else:
                    f = lambda: K.gemm(A, B, out=out, bias=b)  # noqa: E731
            us = t(f)
            f()
            torch.cuda.synchronize()
            res[f"{name}@{M}"] = {"us": round(us, 1), "tflops": round(2 * M * N * Kd / us / 1e6, 1),
                                  "sum": float(out.float().sum())}
            del A, B, out
    print("RESULT " + json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
