"""r03 diagnostic on the 1485dd9 tree with the pre-fix workspace condition: the tiny fp32 flagship step vs the oracle at B = 2, 3, 4
(token counts that are / are not whole 64-row tiles), with every mmfd_gemm decision traced for B = 2."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402
import mmfd  # noqa: E402,F401
from tests.smoke_impl import build_pair, tiny_batch, compare_step  # noqa: E402

for B in (3, 2, 4):
    tr, ref = build_pair("fp32", dropout=0.0)
    if B == 2:
        os.environ["MMFD_TRACE_GEMM"] = "1"
    try:
        compare_step(tr, ref, tiny_batch(B, seed=21), loss_tol=1e-3, grad_rtol=2e-3)
        print("B", B, "ok", flush=True)
    except AssertionError as e:
        print("B", B, "FAIL", "\n".join(x[:100] for x in str(e).split(";")[:12]), flush=True)
    os.environ.pop("MMFD_TRACE_GEMM", None)
