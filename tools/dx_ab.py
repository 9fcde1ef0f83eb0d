"""Same-process timing of the bf16 data-gradient GEMM dY W (+ the GELU-backward epilogue) three ways:
G4 on the transposed weight copy (blocks.linear_dx default), gemm256_kernel on the transposed copy
(G4 off), gemm256_kernel with W as the MN-contiguous operand (trans_b, the round-5 path).
python3 tools/dx_ab.py"""
import os
import sys

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

from mmfd import kernels as K  # noqa: E402

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
    return 1e3 * e0.elapsed_time(e1) / n


for name, M, N, Kd in (("bert ffn2-dx", 65536, 3072, 768), ("vit ffn2-dx", 100864, 3072, 768),
                       ("bert out-dx", 65536, 768, 768), ("vit out-dx", 100864, 768, 768)):
    dy = torch.randn(M, Kd, device=dev).bfloat16()
    W = (torch.randn(Kd, N, device=dev) * 0.05).bfloat16()  # nn.Linear [out, in]
    WT = K.transpose(W)
    for epi in ("plain", "gelu_bwd"):
        if epi == "plain" and "ffn2" in name:
            kw = {}
        elif epi == "gelu_bwd" and "ffn2" in name:
            kw = dict(act=K.ACT_GELU_BWD, aux=torch.randn(M, N, device=dev).bfloat16())
        elif epi == "plain":
            kw = {}
        else:
            continue
        K.set_g4_mode("on")
        g4 = t(lambda: K.gemm(dy, WT, **kw))
        K.set_g4_mode("off")
        g8f = t(lambda: K.gemm(dy, WT, **kw))
        g8t = t(lambda: K.gemm(dy, W, trans_b=True, **kw))
        K.set_g4_mode("on")
        fl = 2.0 * M * N * Kd
        print(f"{name:13s} {epi:8s} G4(W^T) {g4:7.1f} us ({fl / g4 / 1e6:6.1f} TF)  G8(W^T) {g8f:7.1f} us  "
              f"G8(trans_b) {g8t:7.1f} us", flush=True)
