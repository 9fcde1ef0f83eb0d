"""One split-operand GEMM shape (ViT FFN1 forward, operands pre-split) run 5 times, for LDS / MFMA
counter passes: rocprofv3 --pmc SQ_LDS_IDX_ACTIVE ... -- python tools/lds_pmc_gemm.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import mmfd  # noqa: E402,F401
from mmfd import kernels as K  # noqa: E402

M, N, Kd = 100864, 3072, 768
A = torch.randn(M, Kd, device="cuda"); B = torch.randn(N, Kd, device="cuda")
ap, bp = K.split3(A), K.split3(B)
out = torch.empty(M, N, device="cuda")
for _ in range(5):
    K.gemm(A, B, out=out, a_planes=ap, b_planes=bp)
torch.cuda.synchronize()
print("done")
