"""Drop-in mirror of src/model/layers.py (MLP :5-21, MultiHeadAttention :24-58).

Same constructor arguments, sub-module names (MLP.net.0 / net.3) and forward signatures; each
forward is an autograd node over HIP kernels. Inside MisinformationDetectionModel these modules
only hold parameters (the head runs as one fused node, fusion.py); standalone they work as the
reference's layers do.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import blocks as Bk
from . import kernels as K

_COUNT = {"mlp": 0, "mha": 0}


def _next_name(kind):
    """default dropout site of a standalone layer: its kind and construction index ("mlp0",
    "mha1", ...), identical from run to run (a Python object id is not)"""
    n = _COUNT[kind]
    _COUNT[kind] += 1
    return f"{kind}{n}"


class _Seeded:
    """device-resident dropout seed of a standalone layer (manual_seed; advanced by every training
    forward, as the fused model's seeds are)"""

    def manual_seed(self, seed: int):
        self._seed_value = int(seed)
        if getattr(self, "_seed", None) is not None:
            self._seed.set(self._seed_value)
        return self

    def _fork_seed(self, device):
        if getattr(self, "_seed", None) is None or self._seed.t.device != device:
            self._seed = K.Seed(getattr(self, "_seed_value", 0), device=device)
        return self._seed.fork()


class _LinearFn(torch.autograd.Function):
    """y = x W^T + b (nn.Linear) with optional fused GELU and dropout epilogues."""

    @staticmethod
    def forward(ctx, x, w, b, act, p, seed, site):
        shp = x.shape
        x2 = x.reshape(-1, shp[-1]).contiguous()
        wc = w if x.dtype == torch.float32 else K.cast(w, x.dtype)
        aux = torch.empty((x2.shape[0], w.shape[0]), device=x.device, dtype=x.dtype) if act else None
        kw = dict(dropout_p=p, seed=seed, salt=K.salt_of(site)) if p > 0 else {}
        y = K.gemm(x2, wc, bias=b.detach().float().contiguous() if b is not None else None,
                   act=K.ACT_GELU if act else K.ACT_NONE, aux=aux, **kw)
        ctx.save_for_backward(x2, wc, aux)
        ctx.meta = (shp, act, p, seed, site, b is not None)
        return y.reshape(*shp[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, wc, aux = ctx.saved_tensors
        shp, act, p, seed, site, has_b = ctx.meta
        dy2 = dy.reshape(-1, dy.shape[-1]).contiguous().to(x2.dtype)
        if act or p > 0:
            # the epilogue applied dropout after the activation: one elementwise kernel undoes both
            dy2 = K.act_bwd(dy2, aux if act else dy2, K.ACT_GELU if act else K.ACT_NONE, dropout_p=p, seed=seed,
                            salt=K.salt_of(site))
        dx = K.gemm(dy2, wc, trans_b=True).reshape(shp) if ctx.needs_input_grad[0] else None
        db = torch.empty(dy2.shape[1], device=dy2.device, dtype=torch.float32) if has_b else None
        dw = K.gemm(dy2, x2, trans_a=True, trans_b=True, out_dtype=torch.float32, a_rowsum=db)
        return dx, dw, db, None, None, None, None


def linear(x, layer: nn.Linear, act=False, p=0.0, site="", seed=None):
    return _LinearFn.apply(x, layer.weight, layer.bias, act, p, seed if p > 0 else None, site)


class _AttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, Q, Kt, V, H, p, seed, site):
        kw = dict(dropout_p=p, seed=seed, salt=K.salt_of(site)) if p > 0 else {}
        q, k, v = Q.contiguous(), Kt.contiguous(), V.contiguous()
        if kw and Bk.ATTN_DROP_MASK:  # the forward's keep-bitmask, read by the backward (blocks.StepCtx.attn_drop)
            kw["drop_mask"] = K.drop_mask_buffer(q.shape[0], H, q.shape[1], k.shape[1], q.device)
        o, lse = K.attn_fwd(q, k, v, H, **kw)
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.meta = (H, kw)
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        H, kw = ctx.meta
        dq, dk, dv = K.attn_bwd(q, k, v, o, lse, do.contiguous().to(q.dtype), H, **kw)
        return dq, dk, dv, None, None, None, None


class MLP(_Seeded, nn.Module):
    """layers.py:5-21: Linear -> GELU -> Dropout -> Linear -> Dropout. Dropout masks come from the
    counter hash keyed by (seed, site): sites "<name>.h" / "<name>.out" (oracle.fusion_head.mlp)."""

    def __init__(self, embed_dim, mlp_ratio=4.0, dropout=0.1, name=None):
        super().__init__()
        hidden_dim = int(embed_dim * mlp_ratio)
        self.net = nn.Sequential(nn.Linear(embed_dim, hidden_dim), nn.GELU(), nn.Dropout(dropout),
                                 nn.Linear(hidden_dim, embed_dim), nn.Dropout(dropout))
        self.dropout = dropout
        self.site = name or _next_name("mlp")

    def forward(self, x):
        p = self.dropout if self.training else 0.0
        seed = self._fork_seed(x.device) if p > 0 else None
        h = linear(x, self.net[0], act=True, p=p, site=self.site + ".h", seed=seed)
        return linear(h, self.net[3], p=p, site=self.site + ".out", seed=seed)


class MultiHeadAttention(_Seeded, nn.Module):
    """layers.py:24-58: softmax(Q K^T / sqrt(hd)) (no mask), attention dropout, out_proj. The eager
    and `fused_attn` (SDPA) branches are the same computation here (one flash-style kernel).
    Attention-probability dropout site: "<name>.attn" (oracle.fusion_head.mha)."""

    def __init__(self, embed_dim, num_heads, dropout=0.1, fused_attn=False, name=None):
        super().__init__()
        self.embed_dim = embed_dim
        self.num_heads = num_heads
        self.dropout = dropout
        self.fused_attn = fused_attn
        self.attn_dropout = nn.Dropout(dropout)
        self.site = name or _next_name("mha")

    def forward(self, Q, K_, V, out_proj):
        p = self.dropout if self.training else 0.0
        seed = self._fork_seed(Q.device) if p > 0 else None
        ctx = _AttnFn.apply(Q, K_, V, self.num_heads, p, seed, self.site + ".attn")
        if isinstance(out_proj, nn.Linear):
            return linear(ctx, out_proj)
        return out_proj(ctx)
