"""Diagnostic: the tiny flagship step (fp32, split-operand GEMMs, epilogue planes) vs the oracle at
batch sizes whose token counts do / do not allow split-operand weight-gradient GEMMs."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mmfd  # noqa: E402,F401
from tests.smoke_impl import build_pair, tiny_batch, compare_step  # noqa: E402

for B in (2, 3, 4):
    tr, ref = build_pair("fp32", dropout=0.0)
    try:
        compare_step(tr, ref, tiny_batch(B, seed=21), loss_tol=1e-3, grad_rtol=2e-3)
        print("B", B, "ok", flush=True)
    except AssertionError as e:
        print("B", B, "FAIL", "\n".join(x[:80] for x in str(e).split(";")), flush=True)
