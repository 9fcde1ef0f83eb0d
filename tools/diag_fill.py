"""Diagnostic: which host calls launch torch fill / copy kernels during one training step
(torch.profiler with Python stacks; tiny model, the same code path as the bench step)."""
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import mmfd  # noqa: E402,F401
from tests.smoke_impl import build_pair, tiny_batch  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else "bf16"
tr, _ = build_pair(prec, dropout=0.1)
b = {k: v.cuda() for k, v in tiny_batch(3, seed=41).items()}
for _ in range(2):
    tr.step(b)
torch.cuda.synchronize()
with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU], with_stack=True,
                            record_shapes=True) as prof:
    tr.step(b)
    torch.cuda.synchronize()
cnt = collections.Counter()
for ev in prof.events():
    if ev.name in ("aten::fill_", "aten::zero_", "aten::zeros", "aten::copy_", "aten::add_", "aten::clone",
                   "aten::ones", "aten::zeros_like", "aten::add"):
        st = [f for f in (ev.stack or []) if "mmfd" in f or "multimodal" in f or "torch/autograd" in f][:4]
        cnt[(ev.name, " | ".join(st))] += 1
for (n, st), c in cnt.most_common(40):
    print(f"{c:5d} {n:16s} {st}")
