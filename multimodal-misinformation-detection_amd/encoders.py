"""BERT-base text encoder and ViT-B/16 image encoder on HIP kernels (BASELINE configs 2-4).

The reference calls third-party encoders on its hot path (train.py:136-143, preprocess_embeddings.py:
79-92, evaluate.py:129-151) with the HF convention `enc(**inputs).last_hidden_state`. These modules
keep that convention and the hub parameter names (bert-base-uncased / google/vit-base-patch16-224
state_dict names, i.e. transformers 4.47 naming), so pretrained weights load directly. Each encoder
runs as ONE autograd node: forward = embeddings + N layers, backward = hand-written layer backward
over the same kernels (fused QKV GEMM, flash attention with the key-padding mask as an additive
bias, residual adds and dropout in GEMM epilogues, LayerNorm backward with fused residual grads).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import torch
import torch.nn as nn

from . import blocks as Bk
from . import kernels as K


@dataclass
class BertConfig:
    vocab_size: int = 30522
    hidden_size: int = 768
    num_hidden_layers: int = 12
    num_attention_heads: int = 12
    intermediate_size: int = 3072
    max_position_embeddings: int = 512
    type_vocab_size: int = 2
    layer_norm_eps: float = 1e-12
    hidden_dropout_prob: float = 0.1
    attention_probs_dropout_prob: float = 0.1
    pad_token_id: int = 0


@dataclass
class ViTConfig:
    image_size: int = 224
    patch_size: int = 16
    num_channels: int = 3
    hidden_size: int = 768
    num_hidden_layers: int = 12
    num_attention_heads: int = 12
    intermediate_size: int = 3072
    layer_norm_eps: float = 1e-12
    hidden_dropout_prob: float = 0.0
    attention_probs_dropout_prob: float = 0.0


@dataclass
class EncoderOutput:
    last_hidden_state: torch.Tensor
    extra: dict = field(default_factory=dict)


# -------------------------------------------------------------------------------------------------
# BERT
# -------------------------------------------------------------------------------------------------
class BertModel(Bk.CachedWeights, nn.Module):
    """HF BertModel (add_pooling_layer=False) parameter layout; forward returns .last_hidden_state."""

    def __init__(self, config: BertConfig | None = None, **kw):
        super().__init__()
        c = config or BertConfig(**kw)
        self.config = c
        D = c.hidden_size
        self.embeddings = nn.Module()
        self.embeddings.word_embeddings = nn.Embedding(c.vocab_size, D, padding_idx=c.pad_token_id)
        self.embeddings.position_embeddings = nn.Embedding(c.max_position_embeddings, D)
        self.embeddings.token_type_embeddings = nn.Embedding(c.type_vocab_size, D)
        self.embeddings.LayerNorm = nn.LayerNorm(D, eps=c.layer_norm_eps)
        self.encoder = nn.Module()
        self.encoder.layer = nn.ModuleList()
        for _ in range(c.num_hidden_layers):
            L = nn.Module()
            L.attention = nn.Module()
            L.attention.self = nn.Module()
            for n in ("query", "key", "value"):
                setattr(L.attention.self, n, nn.Linear(D, D))
            L.attention.output = nn.Module()
            L.attention.output.dense = nn.Linear(D, D)
            L.attention.output.LayerNorm = nn.LayerNorm(D, eps=c.layer_norm_eps)
            L.intermediate = nn.Module()
            L.intermediate.dense = nn.Linear(D, c.intermediate_size)
            L.output = nn.Module()
            L.output.dense = nn.Linear(c.intermediate_size, D)
            L.output.LayerNorm = nn.LayerNorm(D, eps=c.layer_norm_eps)
            self.encoder.layer.append(L)
        self.compute_dtype = torch.float32
        self._seed = None
        self._seed_value = 0
        self._init_weights()

    def _init_weights(self, std=0.02):
        """HF BertPreTrainedModel._init_weights: N(0, 0.02) linears/embeddings, zero bias, LN 1/0."""
        for m in self.modules():
            if isinstance(m, (nn.Linear, nn.Embedding)):
                nn.init.normal_(m.weight, 0.0, std)
                if isinstance(m, nn.Linear) and m.bias is not None:
                    nn.init.zeros_(m.bias)
                if isinstance(m, nn.Embedding) and m.padding_idx is not None:
                    with torch.no_grad():
                        m.weight[m.padding_idx].zero_()
            elif isinstance(m, nn.LayerNorm):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)

    def set_precision(self, precision):
        self.compute_dtype = {"fp32": torch.float32, "bf16": torch.bfloat16}[precision]
        return self

    def manual_seed(self, seed):
        self._seed_value = int(seed)
        if self._seed is not None:
            self._seed.set(self._seed_value)
        return self

    def _fork_seed(self, dev):
        if self._seed is None or self._seed.t.device != dev:
            self._seed = K.Seed(self._seed_value, device=dev)
        return self._seed.fork()

    def forward(self, input_ids, attention_mask=None, token_type_ids=None, **unused):
        names = [n for n, _ in self.named_parameters()]
        params = [p for _, p in self.named_parameters()]
        if not params[0].is_cuda:
            raise RuntimeError("mmfd BertModel runs on the HIP device: call .to('cuda') first")
        keep = torch.is_grad_enabled() and any(p.requires_grad for p in params)
        out = _BertFn.apply(self, names, keep, input_ids, attention_mask, token_type_ids, *params)
        return EncoderOutput(last_hidden_state=out)


def bert_forward(ctx: Bk.StepCtx, cfg: BertConfig, ids, mask, tts, keep, site="bert"):
    B, L = ids.shape
    D, H = cfg.hidden_size, cfg.num_attention_heads
    eps = cfg.layer_norm_eps
    P = ctx.P
    emb_drop = ctx.drop(site + ".emb")
    s0, x, m0, r0 = K.embed_ln_fwd(ids, tts, P["embeddings.word_embeddings.weight"],
                                   P["embeddings.position_embeddings.weight"],
                                   P["embeddings.token_type_embeddings.weight"], P["embeddings.LayerNorm.weight"],
                                   P["embeddings.LayerNorm.bias"], eps, ctx.dt, **emb_drop)
    kb = K.mask_to_bias(mask) if mask is not None else None
    states = []
    xp = ctx.planes(x) if keep else None  # later layers: from the previous layer's LayerNorm
    for i in range(cfg.num_hidden_layers):
        p = f"encoder.layer.{i}"
        s = f"{site}.L{i}"
        # split-operand fp32 GEMMs: every Linear input is split once (by its producer: LayerNorm,
        # GEMM epilogue, else split3) and the planes are kept for its weight-gradient GEMM (None in
        # bf16 / fp32-MFMA mode)
        qkv = Bk.linear_packed(ctx, x, [p + ".attention.self.query", p + ".attention.self.key",
                                        p + ".attention.self.value"], xp=xp).view(B, L, 3 * D)
        q, k, v = qkv[..., :D], qkv[..., D:2 * D], qkv[..., 2 * D:]
        attn_drop = dict(ctx.attn_drop(s + ".attn", q, k, H)) if cfg.attention_probs_dropout_prob > 0 else {}
        # the output's planes from the attention kernel itself (fp32 split-operand mode)
        op = Bk.new_planes(ctx, B * L, D, q.device) if keep else None
        o, lse = K.attn_fwd(q, k, v, H, key_bias=kb, o_planes=op, **attn_drop)
        s1, _ = Bk.linear(ctx, Bk.as2d(o), p + ".attention.output.dense", residual=x, drop_site=s + ".attn_out",
                          xp=op)
        h1, m1, r1, h1p = Bk.layernorm_planes(ctx, s1, p + ".attention.output.LayerNorm", eps, want=keep)
        T_, I_ = h1.shape[0], cfg.intermediate_size
        # the GELU output feeds only the FFN2 forward and FFN2 weight-gradient GEMMs: its planes come
        # from the FFN1 epilogue, and the fp32 copy is skipped when both run on split operands
        fp, f_out = Bk.out_planes(ctx, T_, I_, [(T_, D, I_), (D, I_, T_, True, True)], h1.device) if keep \
            else (None, True)
        f, pre = Bk.linear(ctx, h1, p + ".intermediate.dense", act=K.ACT_GELU, keep_aux=keep, xp=h1p,
                           out_planes=fp, write_out=f_out)
        s2, _ = Bk.linear(ctx, f, p + ".output.dense", residual=h1, drop_site=s + ".ffn_out", xp=fp)
        x_out, m2, r2, xp_next = Bk.layernorm_planes(ctx, s2, p + ".output.LayerNorm", eps,
                                                     want=keep and i + 1 < cfg.num_hidden_layers)
        if keep:
            states.append((x, qkv, o, lse, s1, m1, r1, h1, pre, f, s2, m2, r2, attn_drop, (xp, op, h1p, fp)))
        x, xp = x_out, xp_next
    st = dict(s0=s0, m0=m0, r0=r0, kb=kb, layers=states, emb_drop=emb_drop) if keep else None
    return x.view(B, L, D), st


def bert_backward(ctx: Bk.StepCtx, cfg: BertConfig, dout, st, ids, tts, site="bert"):
    B, L = ids.shape
    D, H = cfg.hidden_size, cfg.num_attention_heads
    dx = Bk.as2d(dout).contiguous()
    for i in reversed(range(cfg.num_hidden_layers)):
        p = f"encoder.layer.{i}"
        s = f"{site}.L{i}"
        x, qkv, o, lse, s1, m1, r1, h1, pre, f, s2, m2, r2, attn_drop, (xp, op, h1p, fp) = st["layers"][i]
        ds2, ds2d, g2p = Bk.layernorm_bwd_planes(ctx, dx, s2, p + ".output.LayerNorm", m2, r2, drop_site=s + ".ffn_out")
        g2 = ds2d if ds2d is not None else ds2
        ctx.lin_grads([p + ".output.dense"], g2, f, g2p, fp)
        T_, I_ = g2.shape[0], cfg.intermediate_size
        dprep, dpre_out = Bk.out_planes(ctx, T_, I_, [(I_, D, T_, True, True), (T_, D, I_, False, True)], g2.device)
        dpre = Bk.linear_dx(ctx, g2, p + ".output.dense", act=K.ACT_GELU_BWD, aux=pre, dyp=g2p, out_planes=dprep,
                            write_out=dpre_out)
        ctx.lin_grads([p + ".intermediate.dense"], dpre, h1, dprep, h1p)
        # dh1 = ds2 + dpre W (a fresh buffer: the weight-gradient GEMM on the side stream may still be
        # reading ds2)
        dh1 = Bk.linear_dx(ctx, dpre, p + ".intermediate.dense", residual=ds2, dyp=dprep)
        ds1, ds1d, g1p = Bk.layernorm_bwd_planes(ctx, dh1, s1, p + ".attention.output.LayerNorm", m1, r1,
                                                 drop_site=s + ".attn_out")
        g1 = ds1d if ds1d is not None else ds1
        ctx.lin_grads([p + ".attention.output.dense"], g1, Bk.as2d(o), g1p, op)
        do = Bk.linear_dx(ctx, g1, p + ".attention.output.dense", dyp=g1p).view(o.shape)
        dqkv = torch.empty_like(qkv)
        # the packed gradient feeds only the QKV dX / dW GEMMs: planes straight from the attention
        # backward, and no fp32 copy when both run on split operands
        T_ = B * L
        dq2p, dq_out = Bk.out_planes(ctx, T_, 3 * D, [(3 * D, D, T_, True, True), (T_, D, 3 * D, False, True)],
                                     dqkv.device)
        K.attn_bwd(qkv[..., :D], qkv[..., D:2 * D], qkv[..., 2 * D:], o, lse, do, H, key_bias=st["kb"],
                   dq=dqkv[..., :D], dk=dqkv[..., D:2 * D], dv=dqkv[..., 2 * D:], dqkv_planes=dq2p,
                   planes_only=not dq_out, **attn_drop)
        names = [p + ".attention.self.query", p + ".attention.self.key", p + ".attention.self.value"]
        dq2 = Bk.as2d(dqkv)
        dq2._mmfd_planes_only = not dq_out
        ctx.lin_grads(names, dq2, x, dq2p, xp)
        Wp, _ = ctx.w_packed(names)
        dx = Bk.linear_dx(ctx, dq2, Wp, residual=ds1, dyp=dq2p)  # dx_in = ds1 + dQKV [Wq;Wk;Wv] (fresh buffer)
        ctx.flush_ready()
    # embeddings: undo the embedding dropout, LayerNorm backward, scatter into the tables
    if st["emb_drop"]:
        dx = K.dropout(dx, st["emb_drop"]["dropout_p"], st["emb_drop"]["seed"], st["emb_drop"]["salt"])
    dsum, _ = Bk.layernorm_bwd(ctx, dx, st["s0"], "embeddings.LayerNorm", st["m0"], st["r0"])
    P = ctx.P
    z = lambda n: K.zeros(P[n].shape, device=dsum.device)  # noqa: E731  (scatter-add targets)
    dword, dpos, dtyp = (z("embeddings." + n) for n in ("word_embeddings.weight", "position_embeddings.weight",
                                                          "token_type_embeddings.weight"))
    K.embed_bwd(ids, tts, dsum, dword, dpos, dtyp, padding_idx=cfg.pad_token_id)
    ctx.grads["embeddings.word_embeddings.weight"] = dword
    ctx.grads["embeddings.position_embeddings.weight"] = dpos
    ctx.grads["embeddings.token_type_embeddings.weight"] = dtyp
    ctx.flush_ready()


class _BertFn(torch.autograd.Function):
    @staticmethod
    def forward(fctx, model, names, keep, input_ids, attention_mask, token_type_ids, *params):
        cfg = model.config
        P = {n: p.detach() for n, p in zip(names, params)}
        training = model.training
        p = cfg.hidden_dropout_prob if training else 0.0
        if training and cfg.attention_probs_dropout_prob != cfg.hidden_dropout_prob:
            raise NotImplementedError("mmfd BERT uses one dropout probability for hidden and attention dropout")
        dev = params[0].device
        sc = Bk.StepCtx(P, model.compute_dtype, p, model._fork_seed(dev) if training and p > 0 else None,
                        training=training, shadows=Bk.shadow_store(model))
        sc.grad_ready = getattr(model, "_grad_ready", None)
        ids = input_ids.to(dev).long().contiguous()
        B, L = ids.shape
        mask = attention_mask.to(dev).long().contiguous() if attention_mask is not None else None
        tts = token_type_ids.to(dev).long().contiguous() if token_type_ids is not None else None  # None = type 0
        out, st = bert_forward(sc, cfg, ids, mask, tts, keep)
        fctx.keep = keep
        if keep:
            fctx.sc, fctx.st, fctx.model, fctx.names, fctx.ids, fctx.tts = sc, st, model, names, ids, tts
        return out

    @staticmethod
    def backward(fctx, dout):
        sc = fctx.sc
        sc.enable_side_stream(dout.device)
        bert_backward(sc, fctx.model.config, dout.to(sc.dt), fctx.st, fctx.ids, fctx.tts)
        sc.join_side()
        grads = [sc.grads.get(n) for n in fctx.names]
        fctx.sc = fctx.st = None
        return (None, None, None, None, None, None, *grads)


# -------------------------------------------------------------------------------------------------
# ViT
# -------------------------------------------------------------------------------------------------
class ViTModel(Bk.CachedWeights, nn.Module):
    """HF ViTModel (add_pooling_layer=False) with hub parameter names; forward(pixel_values)."""

    def __init__(self, config: ViTConfig | None = None, **kw):
        super().__init__()
        c = config or ViTConfig(**kw)
        self.config = c
        D = c.hidden_size
        npatch = (c.image_size // c.patch_size) ** 2
        self.embeddings = nn.Module()
        self.embeddings.cls_token = nn.Parameter(torch.zeros(1, 1, D))
        self.embeddings.position_embeddings = nn.Parameter(torch.zeros(1, npatch + 1, D))
        self.embeddings.patch_embeddings = nn.Module()
        self.embeddings.patch_embeddings.projection = nn.Conv2d(c.num_channels, D, c.patch_size, c.patch_size)
        self.encoder = nn.Module()
        self.encoder.layer = nn.ModuleList()
        for _ in range(c.num_hidden_layers):
            L = nn.Module()
            L.attention = nn.Module()
            L.attention.attention = nn.Module()
            for n in ("query", "key", "value"):
                setattr(L.attention.attention, n, nn.Linear(D, D))
            L.attention.output = nn.Module()
            L.attention.output.dense = nn.Linear(D, D)
            L.intermediate = nn.Module()
            L.intermediate.dense = nn.Linear(D, c.intermediate_size)
            L.output = nn.Module()
            L.output.dense = nn.Linear(c.intermediate_size, D)
            L.layernorm_before = nn.LayerNorm(D, eps=c.layer_norm_eps)
            L.layernorm_after = nn.LayerNorm(D, eps=c.layer_norm_eps)
            self.encoder.layer.append(L)
        self.layernorm = nn.LayerNorm(D, eps=c.layer_norm_eps)
        self.compute_dtype = torch.float32
        self._init_weights()

    def _init_weights(self, std=0.02):
        for m in self.modules():
            if isinstance(m, (nn.Linear, nn.Conv2d)):
                nn.init.trunc_normal_(m.weight, 0.0, std)
                if m.bias is not None:
                    nn.init.zeros_(m.bias)
            elif isinstance(m, nn.LayerNorm):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
        nn.init.trunc_normal_(self.embeddings.cls_token, 0.0, std)
        nn.init.trunc_normal_(self.embeddings.position_embeddings, 0.0, std)

    def set_precision(self, precision):
        self.compute_dtype = {"fp32": torch.float32, "bf16": torch.bfloat16}[precision]
        return self

    def forward(self, pixel_values, **unused):
        names = [n for n, _ in self.named_parameters()]
        params = [p for _, p in self.named_parameters()]
        if not params[0].is_cuda:
            raise RuntimeError("mmfd ViTModel runs on the HIP device: call .to('cuda') first")
        if self.training and (self.config.hidden_dropout_prob > 0 or self.config.attention_probs_dropout_prob > 0):
            raise NotImplementedError("mmfd ViT supports the ViT-B/16 configuration (dropout 0)")
        keep = torch.is_grad_enabled() and any(p.requires_grad for p in params)
        out = _ViTFn.apply(self, names, keep, pixel_values, *params)
        return EncoderOutput(last_hidden_state=out)


PATCH_W = "embeddings.patch_embeddings.projection.weight"


def vit_forward(ctx: Bk.StepCtx, cfg: ViTConfig, px, keep):
    B = px.shape[0]
    D, H = cfg.hidden_size, cfg.num_attention_heads
    eps = cfg.layer_norm_eps
    P = ctx.P
    patches = K.patchify(px, cfg.patch_size, ctx.dt)
    pe, _ = Bk.linear(ctx, patches, "embeddings.patch_embeddings.projection")
    x = K.vit_tokens_fwd(pe, B, P["embeddings.cls_token"], P["embeddings.position_embeddings"])
    T = x.shape[1]
    x = Bk.as2d(x)
    states = []
    for i in range(cfg.num_hidden_layers):
        p = f"encoder.layer.{i}"
        h, mb, rb, hp = Bk.layernorm_planes(ctx, x, p + ".layernorm_before", eps, want=keep)  # (see BERT)
        qkv = Bk.linear_packed(ctx, h, [p + ".attention.attention.query", p + ".attention.attention.key",
                                        p + ".attention.attention.value"], xp=hp).view(B, T, 3 * D)
        op = Bk.new_planes(ctx, B * T, D, qkv.device) if keep else None
        o, lse = K.attn_fwd(qkv[..., :D], qkv[..., D:2 * D], qkv[..., 2 * D:], H, o_planes=op)
        x1, _ = Bk.linear(ctx, Bk.as2d(o), p + ".attention.output.dense", residual=x, xp=op)
        h2, ma, ra, h2p = Bk.layernorm_planes(ctx, x1, p + ".layernorm_after", eps, want=keep)
        T_, I_ = h2.shape[0], cfg.intermediate_size
        fp, f_out = Bk.out_planes(ctx, T_, I_, [(T_, D, I_), (D, I_, T_, True, True)], h2.device) if keep \
            else (None, True)  # GELU output planes from the FFN1 epilogue (see BERT)
        f, pre = Bk.linear(ctx, h2, p + ".intermediate.dense", act=K.ACT_GELU, keep_aux=keep, xp=h2p,
                           out_planes=fp, write_out=f_out)
        x2, _ = Bk.linear(ctx, f, p + ".output.dense", residual=x1, xp=fp)
        if keep:
            states.append((x, h, mb, rb, qkv, o, lse, x1, h2, ma, ra, pre, f, (hp, op, h2p, fp)))
        x = x2
    y, mf, rf = Bk.layernorm(ctx, x, "layernorm", eps)
    st = dict(patches=patches, layers=states, x_last=x, mf=mf, rf=rf, B=B, T=T) if keep else None
    return y.view(B, T, D), st


def vit_backward(ctx: Bk.StepCtx, cfg: ViTConfig, dout, st):
    D, H = cfg.hidden_size, cfg.num_attention_heads
    dx, _, dxp = Bk.layernorm_bwd_planes(ctx, Bk.as2d(dout).contiguous(), st["x_last"], "layernorm", st["mf"],
                                         st["rf"])
    for i in reversed(range(cfg.num_hidden_layers)):
        p = f"encoder.layer.{i}"
        x, h, mb, rb, qkv, o, lse, x1, h2, ma, ra, pre, f, (hp, op, h2p, fp) = st["layers"][i]
        if dxp is None:
            dxp = ctx.planes(dx)
        ctx.lin_grads([p + ".output.dense"], dx, f, dxp, fp)
        T_, I_ = dx.shape[0], cfg.intermediate_size
        dprep, dpre_out = Bk.out_planes(ctx, T_, I_, [(I_, D, T_, True, True), (T_, D, I_, False, True)], dx.device)
        dpre = Bk.linear_dx(ctx, dx, p + ".output.dense", act=K.ACT_GELU_BWD, aux=pre, dyp=dxp, out_planes=dprep,
                            write_out=dpre_out)
        ctx.lin_grads([p + ".intermediate.dense"], dpre, h2, dprep, h2p)
        dh2 = Bk.linear_dx(ctx, dpre, p + ".intermediate.dense", dyp=dprep)
        dx1, _, dx1p = Bk.layernorm_bwd_planes(ctx, dh2, x1, p + ".layernorm_after", ma, ra, dx_add=dx)
        if dx1p is None:
            dx1p = ctx.planes(dx1)
        ctx.lin_grads([p + ".attention.output.dense"], dx1, Bk.as2d(o), dx1p, op)
        do = Bk.linear_dx(ctx, dx1, p + ".attention.output.dense", dyp=dx1p).view(o.shape)
        dqkv = torch.empty_like(qkv)
        T_ = qkv.shape[0] * qkv.shape[1]  # planes of the packed gradient from the kernels (see BERT)
        dq2p, dq_out = Bk.out_planes(ctx, T_, 3 * D, [(3 * D, D, T_, True, True), (T_, D, 3 * D, False, True)],
                                     dqkv.device)
        K.attn_bwd(qkv[..., :D], qkv[..., D:2 * D], qkv[..., 2 * D:], o, lse, do, H, dq=dqkv[..., :D],
                   dk=dqkv[..., D:2 * D], dv=dqkv[..., 2 * D:], dqkv_planes=dq2p, planes_only=not dq_out)
        names = [p + ".attention.attention.query", p + ".attention.attention.key", p + ".attention.attention.value"]
        dq2 = Bk.as2d(dqkv)
        dq2._mmfd_planes_only = not dq_out
        ctx.lin_grads(names, dq2, h, dq2p, hp)
        Wp, _ = ctx.w_packed(names)
        dh = Bk.linear_dx(ctx, dq2, Wp, dyp=dq2p)
        dx, _, dxp = Bk.layernorm_bwd_planes(ctx, dh, x, p + ".layernorm_before", mb, rb, dx_add=dx1)
        ctx.flush_ready()
    dpatch, dcls, dpos = K.vit_tokens_bwd(dx.view(st["B"], st["T"], D))
    ctx.grads["embeddings.cls_token"] = dcls.view(1, 1, D)
    ctx.grads["embeddings.position_embeddings"] = dpos.view(1, st["T"], D)
    ctx.lin_grads(["embeddings.patch_embeddings.projection"], dpatch, st["patches"])
    ctx.flush_ready()


class _ViTFn(torch.autograd.Function):
    @staticmethod
    def forward(fctx, model, names, keep, pixel_values, *params):
        P = {n: p.detach() for n, p in zip(names, params)}
        P[PATCH_W] = P[PATCH_W].reshape(P[PATCH_W].shape[0], -1)  # conv16/s16 == GEMM over patches
        dev = params[0].device
        sc = Bk.StepCtx(P, model.compute_dtype, 0.0, None, training=model.training, shadows=Bk.shadow_store(model))
        sc.grad_ready = getattr(model, "_grad_ready", None)
        out, st = vit_forward(sc, model.config, pixel_values.to(dev).float().contiguous(), keep)
        fctx.keep = keep
        if keep:
            fctx.sc, fctx.st, fctx.model, fctx.names = sc, st, model, names
            fctx.wshape = params[names.index(PATCH_W)].shape
        return out

    @staticmethod
    def backward(fctx, dout):
        sc = fctx.sc
        sc.enable_side_stream(dout.device)
        vit_backward(sc, fctx.model.config, dout.to(sc.dt), fctx.st)
        sc.join_side()
        sc.grads[PATCH_W] = sc.grads[PATCH_W].view(fctx.wshape)
        grads = [sc.grads.get(n) for n in fctx.names]
        fctx.sc = fctx.st = None
        return (None, None, None, None, *grads)


# -------------------------------------------------------------------------------------------------
# MPNet (the bi-encoder of the evidence corpus: SentenceTransformer("multi-qa-mpnet-base-dot-v1"),
# text2text_retrieval.py:21,125,129-157) — inference only
# -------------------------------------------------------------------------------------------------
@dataclass
class MPNetConfig:
    vocab_size: int = 30527
    hidden_size: int = 768
    num_hidden_layers: int = 12
    num_attention_heads: int = 12
    intermediate_size: int = 3072
    max_position_embeddings: int = 514
    layer_norm_eps: float = 1e-5
    relative_attention_num_buckets: int = 32
    pad_token_id: int = 1


def mpnet_relative_buckets(L, num_buckets=32, max_distance=128):
    """HF MPNetEncoder.relative_position_bucket over arange positions (host, int32 [L, L]); the bucket
    map is a function of L only, computed once per length with the reference's float formula."""
    import math
    ctx_pos = torch.arange(L, dtype=torch.long)[:, None]
    mem_pos = torch.arange(L, dtype=torch.long)[None, :]
    n = -(mem_pos - ctx_pos)
    nb = num_buckets // 2
    ret = (n < 0).to(torch.long) * nb
    n = torch.abs(n)
    max_exact = nb // 2
    is_small = n < max_exact
    large = max_exact + (torch.log(n.float() / max_exact) / math.log(max_distance / max_exact)
                         * (nb - max_exact)).to(torch.long)
    large = torch.min(large, torch.full_like(large, nb - 1))
    ret = ret + torch.where(is_small, n, large)
    return ret.to(torch.int32)


class MPNetModel(Bk.CachedWeights, nn.Module):
    """HF MPNetModel (add_pooling_layer=False) parameter layout; forward(input_ids, attention_mask)
    returns .last_hidden_state. Inference only (the corpus extractor never trains it)."""

    def __init__(self, config: MPNetConfig | None = None, **kw):
        super().__init__()
        c = config or MPNetConfig(**kw)
        self.config = c
        D = c.hidden_size
        self.embeddings = nn.Module()
        self.embeddings.word_embeddings = nn.Embedding(c.vocab_size, D, padding_idx=c.pad_token_id)
        self.embeddings.position_embeddings = nn.Embedding(c.max_position_embeddings, D, padding_idx=c.pad_token_id)
        self.embeddings.LayerNorm = nn.LayerNorm(D, eps=c.layer_norm_eps)
        self.encoder = nn.Module()
        self.encoder.layer = nn.ModuleList()
        for _ in range(c.num_hidden_layers):
            L = nn.Module()
            L.attention = nn.Module()
            L.attention.attn = nn.Module()
            for n in ("q", "k", "v", "o"):
                setattr(L.attention.attn, n, nn.Linear(D, D))
            L.attention.LayerNorm = nn.LayerNorm(D, eps=c.layer_norm_eps)
            L.intermediate = nn.Module()
            L.intermediate.dense = nn.Linear(D, c.intermediate_size)
            L.output = nn.Module()
            L.output.dense = nn.Linear(c.intermediate_size, D)
            L.output.LayerNorm = nn.LayerNorm(D, eps=c.layer_norm_eps)
            self.encoder.layer.append(L)
        self.encoder.relative_attention_bias = nn.Embedding(c.relative_attention_num_buckets, c.num_attention_heads)
        self.compute_dtype = torch.float32
        self._buckets = {}
        self._init_weights()

    def _init_weights(self, std=0.02):
        for m in self.modules():
            if isinstance(m, (nn.Linear, nn.Embedding)):
                nn.init.normal_(m.weight, 0.0, std)
                if isinstance(m, nn.Linear) and m.bias is not None:
                    nn.init.zeros_(m.bias)
                if isinstance(m, nn.Embedding) and m.padding_idx is not None:
                    with torch.no_grad():
                        m.weight[m.padding_idx].zero_()
            elif isinstance(m, nn.LayerNorm):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)

    def set_precision(self, precision):
        self.compute_dtype = {"fp32": torch.float32, "bf16": torch.bfloat16}[precision]
        return self

    def _bucket(self, L, dev):
        key = (L, str(dev))
        b = self._buckets.get(key)
        if b is None:
            b = self._buckets[key] = mpnet_relative_buckets(L, self.config.relative_attention_num_buckets).to(dev)
        return b

    @torch.no_grad()
    def forward(self, input_ids, attention_mask=None, **unused):
        params = dict(self.named_parameters())
        dev = next(iter(params.values())).device
        if dev.type != "cuda":
            raise RuntimeError("mmfd MPNetModel runs on the HIP device: call .to('cuda') first")
        P = {n: p.detach() for n, p in params.items()}
        sc = Bk.StepCtx(P, self.compute_dtype, shadows=Bk.shadow_store(self))
        ids = input_ids.to(dev).long().contiguous()
        mask = attention_mask.to(dev).long().contiguous() if attention_mask is not None else None
        out = mpnet_forward(sc, self.config, ids, mask, self._bucket(ids.shape[1], dev))
        return EncoderOutput(last_hidden_state=out)


def mpnet_forward(ctx: Bk.StepCtx, cfg: MPNetConfig, ids, mask, bucket):
    B, L = ids.shape
    D, H = cfg.hidden_size, cfg.num_attention_heads
    eps = cfg.layer_norm_eps
    P = ctx.P
    pos_ids = K.position_ids(ids, cfg.pad_token_id)
    x = K.embed_ln_infer(ids, pos_ids, P["embeddings.word_embeddings.weight"],
                         P["embeddings.position_embeddings.weight"], P["embeddings.LayerNorm.weight"],
                         P["embeddings.LayerNorm.bias"], eps, ctx.dt)
    kb = K.mask_to_bias(mask) if mask is not None else None
    rb = K.rel_bias(bucket, P["encoder.relative_attention_bias.weight"])
    for i in range(cfg.num_hidden_layers):
        p = f"encoder.layer.{i}"
        qkv = Bk.linear_packed(ctx, x, [p + ".attention.attn.q", p + ".attention.attn.k",
                                        p + ".attention.attn.v"]).view(B, L, 3 * D)
        o, _ = K.attn_fwd(qkv[..., :D], qkv[..., D:2 * D], qkv[..., 2 * D:], H, key_bias=kb, rel_bias=rb)
        s1, _ = Bk.linear(ctx, Bk.as2d(o), p + ".attention.attn.o", residual=x)
        h1, _, _ = Bk.layernorm(ctx, s1, p + ".attention.LayerNorm", eps)
        f, _ = Bk.linear(ctx, h1, p + ".intermediate.dense", act=K.ACT_GELU)
        s2, _ = Bk.linear(ctx, f, p + ".output.dense", residual=h1)
        x, _, _ = Bk.layernorm(ctx, s2, p + ".output.LayerNorm", eps)
    return x.view(B, L, D)
