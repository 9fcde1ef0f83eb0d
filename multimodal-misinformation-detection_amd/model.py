"""Drop-in mirror of the reference fusion model (src/model/model.py:6-468).

Same classes, constructor arguments, forward signatures, return structure and state_dict names as
the reference (108 entries in the 4-path mode, model.py:19-53, 137-170, 252-288), so checkpoints
saved by the reference's train.py (`model_state_dict`) load unchanged. The sub-modules only hold
parameters: `MisinformationDetectionModel.forward` runs the whole head as ONE autograd node whose
forward and backward are sequences of HIP kernels (fusion.py).

Precision: `model.compute_dtype` (torch.float32 = parity mode, default; torch.bfloat16 =
throughput mode, bf16 operands with fp32 accumulation, fp32 master weights and gradients).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import blocks as Bk
from . import fusion as FU
from . import kernels as K
from .layers import MLP, MultiHeadAttention


class MultiViewClaimRepresentation(nn.Module):
    """model.py:6-121 (parameters only; computed by fusion.py)."""

    def __init__(self, text_input_dim=768, image_input_dim=1024, embed_dim=256, num_heads=8, dropout=0.1,
                 mlp_ratio=4.0, fused_attn=False):
        super().__init__()
        self.text_input_dim, self.image_input_dim = text_input_dim, image_input_dim
        self.embed_dim, self.num_heads, self.dropout = embed_dim, num_heads, dropout
        self.text_proj = nn.Linear(text_input_dim, embed_dim)
        self.image_proj = nn.Linear(image_input_dim, embed_dim)
        self.text_WQ = nn.Linear(embed_dim, embed_dim)
        self.text_WK = nn.Linear(embed_dim, embed_dim)
        self.text_WV = nn.Linear(embed_dim, embed_dim)
        self.image_WQ = nn.Linear(embed_dim, embed_dim)
        self.image_WK = nn.Linear(embed_dim, embed_dim)
        self.image_WV = nn.Linear(embed_dim, embed_dim)
        self.text_self_attn_out = nn.Linear(embed_dim, embed_dim)
        self.image_self_attn_out = nn.Linear(embed_dim, embed_dim)
        self.text_cross_attn_out = nn.Linear(embed_dim, embed_dim)
        self.image_cross_attn_out = nn.Linear(embed_dim, embed_dim)
        self.text_self_ln1 = nn.LayerNorm(embed_dim)
        self.text_self_ln2 = nn.LayerNorm(embed_dim)
        self.image_self_ln1 = nn.LayerNorm(embed_dim)
        self.image_self_ln2 = nn.LayerNorm(embed_dim)
        self.text_cross_ln1 = nn.LayerNorm(embed_dim)
        self.text_cross_ln2 = nn.LayerNorm(embed_dim)
        self.image_cross_ln1 = nn.LayerNorm(embed_dim)
        self.image_cross_ln2 = nn.LayerNorm(embed_dim)
        self.text_mlp = MLP(embed_dim, mlp_ratio, dropout)
        self.image_mlp = MLP(embed_dim, mlp_ratio, dropout)
        self.attention = MultiHeadAttention(embed_dim, num_heads, dropout, fused_attn)
        self.proj_dropout = nn.Dropout(dropout)


class CrossAttentionEvidenceConditioning(nn.Module):
    """model.py:124-237 (parameters only)."""

    def __init__(self, text_input_dim=768, image_input_dim=1024, embed_dim=256, num_heads=8, dropout=0.1,
                 mlp_ratio=4.0, fused_attn=False):
        super().__init__()
        self.num_heads, self.embed_dim, self.dropout, self.fused_attn = num_heads, embed_dim, dropout, fused_attn
        self.text_WQ = nn.Linear(embed_dim, embed_dim)
        self.image_WQ = nn.Linear(embed_dim, embed_dim)
        self.text_evidence_key = nn.Linear(text_input_dim, embed_dim)
        self.text_evidence_value = nn.Linear(text_input_dim, embed_dim)
        self.image_evidence_key = nn.Linear(image_input_dim, embed_dim)
        self.image_evidence_value = nn.Linear(image_input_dim, embed_dim)
        self.text_text_out = nn.Linear(embed_dim, embed_dim)
        self.text_image_out = nn.Linear(embed_dim, embed_dim)
        self.image_text_out = nn.Linear(embed_dim, embed_dim)
        self.image_image_out = nn.Linear(embed_dim, embed_dim)
        for n in ("text_text", "text_image", "image_text", "image_image"):
            setattr(self, f"{n}_ln1", nn.LayerNorm(embed_dim))
            setattr(self, f"{n}_ln2", nn.LayerNorm(embed_dim))
        self.text_mlp = MLP(embed_dim, mlp_ratio, dropout)
        self.image_mlp = MLP(embed_dim, mlp_ratio, dropout)
        self.attention = MultiHeadAttention(embed_dim, num_heads, dropout, fused_attn)
        self.proj_dropout = nn.Dropout(dropout)


def _cls_head(in_dim, hidden_dims, num_classes, dropout):
    layers = []
    d = in_dim
    for h in hidden_dims:
        layers += [nn.Linear(d, h), nn.ReLU(), nn.Dropout(dropout)]
        d = h
    layers.append(nn.Linear(d, num_classes))
    return nn.Sequential(*layers)


class ClassificationModule(nn.Module):
    """model.py:240-347 (parameters only)."""

    def __init__(self, embed_dim=256, hidden_dim=64, num_classes=3, dropout=0.1, factify=False):
        super().__init__()
        self.factify = factify
        if factify:
            self.unified_mlp = _cls_head(embed_dim * 4, [hidden_dim * 2, hidden_dim], num_classes, dropout)
        else:
            self.mlp_text_given_text = _cls_head(embed_dim, [hidden_dim], num_classes, dropout)
            self.mlp_text_given_image = _cls_head(embed_dim, [hidden_dim], num_classes, dropout)
            self.mlp_image_given_text = _cls_head(embed_dim, [hidden_dim], num_classes, dropout)
            self.mlp_image_given_image = _cls_head(embed_dim, [hidden_dim], num_classes, dropout)


class _HeadFn(torch.autograd.Function):
    """The whole fusion head as one autograd node (forward: fusion.head_forward, backward:
    fusion.head_backward). Outputs: (y_tt, y_ti, y_it, y_ii) or (pred,) — None for absent paths.
    With `pairs_B` > 0 the text / image inputs are the STACKED encoder outputs [2B, L, D] of
    FusionTrainer (claims rows [:B], evidence rows [B:]): the backward then writes dX and dE into
    the two halves of one gradient buffer per modality instead of two slice-backward scatters."""

    @staticmethod
    def forward(ctx, model, pairs_B, X_t, X_i, E_t, E_i, *params):
        names = model._param_names
        P = {n: p.detach() for n, p in zip(names, params)}
        sc = Bk.StepCtx(P, model.compute_dtype, model.dropout_p, model._get_seed() if model.training else None,
                        training=model.training, shadows=Bk.shadow_store(model))
        sc.grad_ready = getattr(model, "_grad_ready", None)
        ctx.pairs_B = pairs_B
        ctx.stacked = [None if x is None else (x.shape, x.dtype) for x in (X_t, X_i)] if pairs_B else None
        if pairs_B:
            (T, I), B = (X_t, X_i), pairs_B
            X_t, E_t = (T[:B], T[B:]) if T is not None else (None, None)
            X_i, E_i = (I[:B], I[B:]) if I is not None else (None, None)
        outs, state = FU.head_forward(sc, model._cfg, X_t, X_i, E_t, E_i)
        ctx.sc, ctx.state, ctx.model = sc, state, model
        ctx.in_shapes = [None if x is None else (x.shape, x.dtype) for x in (X_t, X_i, E_t, E_i)]
        if model._cfg.factify or model._cfg.text_only:
            ctx.tags = ["pred"]
            ctx.out_shapes = [outs["pred"].shape]
            return outs["pred"], None, None, None
        ctx.tags = ["tt", "ti", "it", "ii"]
        ctx.out_shapes = [outs[t].shape if t in outs else None for t in ctx.tags]
        return tuple(outs.get(t) for t in ctx.tags)

    @staticmethod
    def backward(ctx, *grads):
        sc, state, model = ctx.sc, ctx.state, ctx.model
        douts = {}
        for t, g, shp in zip(ctx.tags, grads, ctx.out_shapes):
            if shp is None:
                continue
            douts[t] = g.contiguous().float() if g is not None else torch.zeros(shp, device=state["S"][
                next(iter(state["S"]))].device, dtype=torch.float32)
        need = ctx.needs_input_grad
        if ctx.pairs_B:
            B = ctx.pairs_B
            bufs, outs = [], []
            for i, st in enumerate(ctx.stacked):
                if st is None or not need[2 + i]:
                    bufs.append(None)
                    outs += [None, None]
                    continue
                buf = torch.empty(st[0], device=douts[ctx.tags[0]].device, dtype=st[1])
                bufs.append(buf)
                direct = st[1] == sc.dt  # the GEMMs write the halves directly
                outs += [Bk.as2d(buf[:B]) if direct else None, Bk.as2d(buf[B:]) if direct else None]
            nt, ni = bufs[0] is not None, bufs[1] is not None
            dXt, dXi, dEt, dEi = FU.head_backward(sc, model._cfg, douts, state, need_dX=(nt, ni), need_dE=(nt, ni),
                                                  outs=(outs[0], outs[2], outs[1], outs[3]))
            sc.flush_ready()
            for buf, (a, b), (oa, ob) in zip(bufs, ((dXt, dEt), (dXi, dEi)), ((outs[0], outs[1]), (outs[2], outs[3]))):
                if buf is None:
                    continue
                for d, o, half in ((a, oa, buf[:B]), (b, ob, buf[B:])):
                    if d is None:  # no path consumed these rows (text_only / unimodal heads)
                        K.zero_(half)
                    elif o is None:  # compute dtype differs from the encoders' output dtype
                        K.cast(d.contiguous(), buf.dtype, out=half)
            pgrads = [sc.grads.get(n) for n in model._param_names]
            ctx.sc = ctx.state = None
            return (None, None, bufs[0], bufs[1], None, None, *pgrads)
        dXt, dXi, dEt, dEi = FU.head_backward(sc, model._cfg, douts, state, need_dX=(need[2], need[3]),
                                              need_dE=(need[4], need[5]))
        sc.flush_ready()

        def back(d, shp):
            if d is None or shp is None:
                return None
            return d if d.dtype == shp[1] else K.cast(d, shp[1])

        dxs = [back(d, s) if need[i + 2] else None for i, (d, s) in enumerate(zip((dXt, dXi, dEt, dEi),
                                                                                   ctx.in_shapes))]
        pgrads = [sc.grads.get(n) for n in model._param_names]
        ctx.sc = ctx.state = None
        return (None, None, *dxs, *pgrads)


class MisinformationDetectionModel(Bk.CachedWeights, nn.Module):
    """model.py:350-468. forward(X_t, X_i, E_t, E_i) -> ((y_tt, y_ti), (y_it, y_ii)) or (pred, None)."""

    def __init__(self, text_input_dim=768, image_input_dim=1024, embed_dim=256, num_heads=8, dropout=0.1,
                 hidden_dim=64, num_classes=3, mlp_ratio=4.0, fused_attn=False, factify=False, text_only=False):
        super().__init__()
        self.factify = factify
        self.text_only = text_only
        self.representation = MultiViewClaimRepresentation(text_input_dim, image_input_dim, embed_dim, num_heads,
                                                           dropout, mlp_ratio, fused_attn)
        self.cross_attn = CrossAttentionEvidenceConditioning(text_input_dim, image_input_dim, embed_dim, num_heads,
                                                             dropout, mlp_ratio, fused_attn)
        if text_only:
            self.text_classifier = _cls_head(embed_dim, [hidden_dim * 2, hidden_dim], num_classes, dropout)
        else:
            self.classifier = ClassificationModule(embed_dim, hidden_dim, num_classes, dropout, factify)
        self._initialize_weights()
        self.compute_dtype = torch.float32
        self.dropout_p = float(dropout)
        self._cfg = FU.HeadConfig(embed_dim, num_heads, factify=factify, text_only=text_only)
        self._seed = None
        self._seed_value = 0

    def _initialize_weights(self):
        """model.py:416-424"""
        for module in self.modules():
            if isinstance(module, nn.Linear):
                nn.init.xavier_uniform_(module.weight)
                if module.bias is not None:
                    nn.init.zeros_(module.bias)
            elif isinstance(module, nn.LayerNorm):
                nn.init.ones_(module.weight)
                nn.init.zeros_(module.bias)

    # ---- mmfd extensions ---------------------------------------------------------------------------
    def set_precision(self, precision: str):
        self.compute_dtype = {"fp32": torch.float32, "bf16": torch.bfloat16}[precision]
        return self

    def manual_seed(self, seed: int):
        """Seed of the counter-based dropout masks (advanced by one every training forward)."""
        self._seed_value = int(seed)
        if self._seed is not None:
            self._seed.set(self._seed_value)
        return self

    def _get_seed(self):
        dev = next(self.parameters()).device
        if self._seed is None or self._seed.t.device != dev:
            self._seed = K.Seed(self._seed_value, device=dev)
        return self._seed.fork()

    @property
    def _param_names(self):
        return [n for n, _ in self.named_parameters()]

    def forward(self, X_t=None, X_i=None, E_t=None, E_i=None):
        params = [p for _, p in self.named_parameters()]
        if not params[0].is_cuda:
            raise RuntimeError("mmfd MisinformationDetectionModel runs on the HIP device: call .to('cuda') first")
        outs = _HeadFn.apply(self, 0, X_t, X_i, E_t, E_i, *params)
        if self.factify or self.text_only:
            return outs[0], None
        return (outs[0], outs[1]), (outs[2], outs[3])

    def forward_pairs(self, T, I, B):
        """forward(T[:B], I[:B], T[B:], I[B:]) on stacked claim/evidence encoder outputs (T / I
        [2B, L, D]); their gradients come back as one tensor each (FusionTrainer)."""
        params = [p for _, p in self.named_parameters()]
        if not params[0].is_cuda:
            raise RuntimeError("mmfd MisinformationDetectionModel runs on the HIP device: call .to('cuda') first")
        outs = _HeadFn.apply(self, int(B), T, I, None, None, *params)
        if self.factify or self.text_only:
            return outs[0], None
        return (outs[0], outs[1]), (outs[2], outs[3])
