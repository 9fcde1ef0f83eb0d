import os, sys, collections
sys.path.insert(0, os.getcwd())
import torch
import mmfd
from mmfd.train import build_flagship
from mmfd.dataset import synthetic_batch
tr = build_flagship("cuda", sys.argv[1] if len(sys.argv) > 1 else "bf16")
b = synthetic_batch(8, device="cuda")
tr.step(b); tr.step(b); torch.cuda.synchronize()
from torch.profiler import profile, ProfilerActivity
with profile(activities=[ProfilerActivity.CPU], with_stack=True, record_shapes=True) as prof:
    tr.step(b); torch.cuda.synchronize()
c = collections.Counter()
for e in prof.events():
    if e.name in ("aten::fill_", "aten::zero_", "aten::zeros", "aten::zeros_like", "aten::copy_", "aten::_to_copy"):
        st = [s for s in (e.stack or []) if "mmfd" in s or "multimodal" in s or "torch/autograd" in s or "torch/optim" in s][:3]
        c[(e.name, tuple(st), str(e.input_shapes)[:60])] += 1
for k, v in c.most_common(25):
    print(v, k)
