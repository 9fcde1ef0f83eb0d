"""Times the deterministic embedding backward (csrc/embed_bwd.hip) alone on the bench's BERT shape:
512 sequences x 128 tokens x 768, synthetic_batch ids ([CLS] / [SEP] in every row), bf16 and fp32,
HIP events around N calls on one stream. Run on the GPU box: python tools/embed_bench.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mmfd  # noqa: E402
from mmfd import kernels as K  # noqa: E402
from mmfd.dataset import synthetic_batch  # noqa: E402


def main():
    it = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    b = synthetic_batch(256, seed=1000, device="cuda")
    ids = b["input_ids"]
    tts = torch.zeros_like(ids)
    B, L = ids.shape
    D, V = 768, 30522
    for dt in (torch.bfloat16, torch.float32):
        dsum = torch.randn(B, L, D, device="cuda").to(dt)
        dword = torch.zeros(V, D, device="cuda")
        dpos = torch.zeros(512, D, device="cuda")
        dtyp = torch.zeros(2, D, device="cuda")
        for _ in range(3):
            K.embed_bwd(ids, tts, dsum, dword, dpos, dtyp, padding_idx=0)
        torch.cuda.synchronize()
        for name, args in (("all three tables", (dword, dpos[:L], dtyp)), ("word only", (dword, None, None)),
                           ("position only", (None, dpos[:L], None)), ("type only", (None, None, dtyp))):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(it):
                K.embed_bwd(ids, tts, dsum, *args, padding_idx=0)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / it
            gb = B * L * D * dsum.element_size() / 1e9
            print(f"{str(dt):15s} {name:17s} {us:8.1f} us/call  ({gb / us * 1e6 / 1e3:.2f} TB/s of dsum reads)")
    print("mmfd", mmfd.__version__ if hasattr(mmfd, "__version__") else "")


if __name__ == "__main__":
    main()
