"""Run one bf16 GEMM shape a few times (for rocprofv3 counter passes).
python tools/gemm_one.py M N K [layout nt|nn|tn] [iters]"""
import os
import sys

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

import mmfd  # noqa: E402,F401
from mmfd import kernels as K  # noqa: E402

M, N, Kd = (int(x) for x in sys.argv[1:4])
layout = sys.argv[4] if len(sys.argv) > 4 else "nt"
iters = int(sys.argv[5]) if len(sys.argv) > 5 else 5
A = torch.randn(M, Kd, device="cuda").bfloat16()
B = torch.randn(N, Kd, device="cuda").bfloat16()
kw = {}
if layout in ("nn", "tn"):
    B = B.T.contiguous(); kw["trans_b"] = True
if layout == "tn":
    A = A.T.contiguous(); kw["trans_a"] = True
out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
for _ in range(iters):
    K.gemm(A, B, out=out, alpha=float(os.environ.get("ALPHA", "1.0")), **kw)
torch.cuda.synchronize()
print("ok")
