"""Times the four-wave GEMM (MMFD_G4_KMAX=4096: every K) against gemm256_kernel (MMFD_G4=0) on the
step's forward products, for the library MMFD_LIB_PATH points at (tools/g4_variant.sh builds the
schedule variants); also checks the two are bit-identical."""
import os
import sys

os.environ["MMFD_G4_KMAX"] = "4096"
sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

import mmfd.kernels as K  # noqa: E402

dev = torch.device("cuda", 0)
tag = os.path.basename(os.path.dirname(os.environ.get("MMFD_LIB_PATH", "in-tree/x")))
seed = K.Seed(99, device=dev)
tot = {"1": 0.0, "0": 0.0}
for name, M, N, Kd, mode in (("bert qkv", 65536, 2304, 768, "bias"), ("vit ffn1 gelu", 100864, 3072, 768, "gelu"),
                             ("bert out drop+res", 65536, 768, 768, "dropres"),
                             ("bert ffn2 drop+res", 65536, 768, 3072, "dropres"), ("vit ffn2 res", 100864, 768, 3072, "res")):
    g = torch.Generator(device=dev).manual_seed(M + N)
    A = torch.randn(M, Kd, device=dev, generator=g).bfloat16(); B = torch.randn(N, Kd, device=dev, generator=g).bfloat16()
    kw = dict(bias=torch.randn(N, device=dev, generator=g))
    if mode == "gelu":
        kw.update(act=K.ACT_GELU, aux=torch.empty(M, N, device=dev, dtype=torch.bfloat16))
    elif mode == "dropres":
        kw.update(residual=torch.randn(M, N, device=dev, generator=g).bfloat16(), dropout_p=0.1, seed=seed, salt=3)
    elif mode == "res":
        kw.update(residual=torch.randn(M, N, device=dev, generator=g).bfloat16())
    res = {}
    for g4 in ("1", "0"):
        K.set_g4_mode("on" if g4 == "1" else "off")
        for _ in range(3):
            out = K.gemm(A, B, **kw)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            out = K.gemm(A, B, **kw)
        e1.record()
        torch.cuda.synchronize()
        res[g4] = (e0.elapsed_time(e1) / 20 * 1e3, out.clone())
        tot[g4] += res[g4][0]
    same = torch.equal(res["1"][1], res["0"][1])
    print(f"{tag:6s} {name:20s} g4 {res['1'][0]:7.1f} us  g8 {res['0'][0]:7.1f} us  ({res['0'][0] / res['1'][0]:.3f}x)  "
          f"bit-identical: {same}", flush=True)
print(f"{tag:6s} sum g4 {tot['1']:.1f} us  g8 {tot['0']:.1f} us", flush=True)
