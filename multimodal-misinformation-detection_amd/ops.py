"""Fake (meta) kernels of the torch.ops.mmfd custom ops registered by libmmfd_torch.so
(csrc/torch_ops.cpp), so the ops trace under FakeTensorMode / torch.compile / the meta device:
the out-variant ops (the C ABI never allocates) only mutate their declared out arguments and
return nothing; `mmfd::linear` returns its [..., N] output. Imported by mmfd.kernels.load()."""
from __future__ import annotations

import torch

_OUT_VARIANT = ("gemm", "attn_fwd", "attn_bwd", "layernorm_fwd", "layernorm_bwd", "xent", "adamw", "seq_mean_fwd",
                "seq_mean_bwd", "cast", "cosine_scores", "topk", "split3")


def _noop(*args, **kwargs):
    return None


for _name in _OUT_VARIANT:
    torch.library.register_fake(f"mmfd::{_name}")(_noop)


@torch.library.register_fake("mmfd::linear")
def _linear_fake(x, w, bias=None, act=0):
    torch._check(x.shape[-1] == w.shape[1], lambda: "mmfd::linear: inner dims differ")
    return x.new_empty((*x.shape[:-1], w.shape[0]))
