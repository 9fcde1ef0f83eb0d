"""DeBERTa-v3 text encoder on HIP kernels — the reference's default text encoder
(`AutoModel.from_pretrained("microsoft/deberta-v3-xsmall")`, train.py:330-331, called with
`.last_hidden_state` at train.py:136-140, preprocess_embeddings.py:63-80, evaluate.py:112-132).

HF parameter names (a hub / transformers state_dict loads unchanged) and HF's arithmetic
(transformers modeling_deberta_v2.py, restated in oracle/deberta.py): word embedding -> LayerNorm
-> times the mask; per layer the disentangled self-attention

    S = Q (K / sqrt(3 d))^T + c2p[i, clamp(rel(i,j) + 256)] / sqrt(3 d) + p2c[j, clamp(-rel(j,i) + 256)] / sqrt(3 d)

with c2p = Q_h . posK_h^T, p2c = K_h . posQ_h^T, posQ|posK = the layer's own Q/K projections of
LayerNorm(rel_embeddings) (share_att_key), rel = log-bucket relative positions (256 buckets,
max 512); padded keys masked with finfo.min; a fully padded query row averages V over all keys
(masked_fill + softmax semantics). Then the post-LN BERT block (out proj + residual + LN, GELU
FFN + residual + LN).

MI355X mapping: QKV is one packed GEMM; the position projections of all heads are one GEMM of the
512 relative embeddings against the same packed weight; c2p / p2c are per-head MFMA GEMMs
([B*L, d] x [d, 512]); one gather kernel turns them into the [B, H, L, L] fp32 additive bias the
flash-attention kernels consume (batch-strided rel_bias); padded-row fix-ups are two tiny kernels.
Inference only (the reference freezes its encoders, train.py:335-340, and the pre-embedding
pass runs under no_grad): a forward that would need gradients raises.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch
import torch.nn as nn

from . import blocks as Bk
from . import kernels as K
from .encoders import EncoderOutput


@dataclass
class DebertaV2Config:
    """microsoft/deberta-v3-xsmall defaults (relative_attention, share_att_key, pos_att_type
    p2c|c2p, norm_rel_ebd layer_norm, position_biased_input False, type_vocab_size 0 are fixed)."""
    vocab_size: int = 128100
    hidden_size: int = 384
    num_hidden_layers: int = 12
    num_attention_heads: int = 6
    intermediate_size: int = 1536
    max_position_embeddings: int = 512
    position_buckets: int = 256
    max_relative_positions: int = -1
    layer_norm_eps: float = 1e-7
    pad_token_id: int = 0


def log_bucket_relative_positions(L: int, bucket_size: int, max_position: int) -> np.ndarray:
    """rel[i, j] = make_log_bucket_position(i - j, bucket_size, max_position) (modeling_deberta_v2.py:57-95),
    computed on the host in float64 like torch's float path, int64 [L, L]"""
    rel = (np.arange(L)[:, None] - np.arange(L)[None, :]).astype(np.int64)
    if bucket_size <= 0 or max_position <= 0:
        return rel
    mid = bucket_size // 2
    sign = np.sign(rel)
    abs_pos = np.where((rel < mid) & (rel > -mid), mid - 1, np.abs(rel)).astype(np.float32)
    log_pos = np.ceil(np.log(abs_pos / np.float32(mid)) / np.log(np.float32((max_position - 1) / mid))
                      * np.float32(mid - 1)).astype(np.float32) + mid
    return np.where(abs_pos <= mid, rel.astype(np.float32), log_pos * sign).astype(np.int64)


_IDX = {}


def _bias_indices(L, S, max_position, device):
    """int32 [L, L] c2p and p2c gather indices: clamp(rel + S) and clamp(-rel + S) (:323, :339)"""
    key = (L, S, max_position, str(device))
    t = _IDX.get(key)
    if t is None:
        rel = log_bucket_relative_positions(L, S, max_position)
        c2p = np.clip(rel + S, 0, 2 * S - 1).astype(np.int32)
        p2c = np.clip(-rel + S, 0, 2 * S - 1).astype(np.int32)
        t = _IDX[key] = (torch.from_numpy(c2p).to(device), torch.from_numpy(p2c).to(device))
    return t


class DebertaV2Model(Bk.CachedWeights, nn.Module):
    def __init__(self, config: DebertaV2Config | None = None, **kw):
        super().__init__()
        c = config or DebertaV2Config(**kw)
        self.config = c
        D, I = c.hidden_size, c.intermediate_size
        self.embeddings = nn.Module()
        self.embeddings.word_embeddings = nn.Embedding(c.vocab_size, D, padding_idx=c.pad_token_id)
        self.embeddings.LayerNorm = nn.LayerNorm(D, eps=c.layer_norm_eps)
        self.encoder = nn.Module()
        self.encoder.layer = nn.ModuleList()
        for _ in range(c.num_hidden_layers):
            L = nn.Module()
            L.attention = nn.Module()
            L.attention.self = nn.Module()
            for n in ("query_proj", "key_proj", "value_proj"):
                setattr(L.attention.self, n, nn.Linear(D, D))
            L.attention.output = nn.Module()
            L.attention.output.dense = nn.Linear(D, D)
            L.attention.output.LayerNorm = nn.LayerNorm(D, eps=c.layer_norm_eps)
            L.intermediate = nn.Module()
            L.intermediate.dense = nn.Linear(D, I)
            L.output = nn.Module()
            L.output.dense = nn.Linear(I, D)
            L.output.LayerNorm = nn.LayerNorm(D, eps=c.layer_norm_eps)
            self.encoder.layer.append(L)
        self.encoder.rel_embeddings = nn.Embedding(2 * self.att_span, D)
        self.encoder.LayerNorm = nn.LayerNorm(D, eps=c.layer_norm_eps)
        self.compute_dtype = torch.float32
        self._zero_pos = {}
        self._init_weights()

    @property
    def att_span(self):
        c = self.config
        mrp = c.max_relative_positions if c.max_relative_positions > 0 else c.max_position_embeddings
        return c.position_buckets if c.position_buckets > 0 else mrp

    @property
    def max_relative_positions(self):
        c = self.config
        return c.max_relative_positions if c.max_relative_positions > 0 else c.max_position_embeddings

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

    def forward(self, input_ids, attention_mask=None, token_type_ids=None, **unused):
        params = dict(self.named_parameters())
        first = next(iter(params.values()))
        if not first.is_cuda:
            raise RuntimeError("mmfd DebertaV2Model runs on the HIP device: call .to('cuda') first")
        if torch.is_grad_enabled() and any(p.requires_grad for p in params.values()):
            raise NotImplementedError("mmfd DebertaV2Model is inference-only (frozen encoder, train.py:335-340): "
                                      "call it under torch.no_grad() or freeze its parameters")
        P = {n: p.detach() for n, p in params.items()}
        ctx = Bk.StepCtx(P, self.compute_dtype, shadows=Bk.shadow_store(self))
        ctx.cache_derived = True          # frozen encoder: packed QKV biases persist across calls
        out = deberta_forward(self, ctx, input_ids, attention_mask)
        return EncoderOutput(last_hidden_state=out)


def deberta_forward(model: DebertaV2Model, ctx: Bk.StepCtx, input_ids, attention_mask):
    cfg = model.config
    dev = ctx.P["embeddings.word_embeddings.weight"].device
    ids = input_ids.to(dev).long().contiguous()
    B, L = ids.shape
    mask = (attention_mask.to(dev).long().contiguous() if attention_mask is not None else torch.ones_like(ids))
    D, H = cfg.hidden_size, cfg.num_attention_heads
    d = D // H
    S = model.att_span
    eps = cfg.layer_norm_eps
    dt = ctx.dt
    # embeddings: LN(word[id]) * mask (no absolute positions, no token types)
    zp = model._zero_pos.get((L, str(dev)))
    if zp is None:
        zp = model._zero_pos[(L, str(dev))] = torch.zeros(L, D, device=dev, dtype=torch.float32)
    x = K.embed_ln_infer(ids, None, ctx.P["embeddings.word_embeddings.weight"], zp,
                         ctx.P["embeddings.LayerNorm.weight"], ctx.P["embeddings.LayerNorm.bias"], eps, dt)
    K.mask_rows(x, mask)
    key_bias = K.mask_to_bias(mask)
    c2p_idx, p2c_idx = _bias_indices(L, S, model.max_relative_positions, dev)
    rel = ctx.P["encoder.rel_embeddings.weight"][: 2 * S]
    relE, _, _ = K.layernorm_fwd(K.cast(rel, dt) if dt != torch.float32 else rel.contiguous(),
                                 ctx.P["encoder.LayerNorm.weight"], ctx.P["encoder.LayerNorm.bias"], eps)
    scale = 1.0 / math.sqrt(d * 3)
    c2p = torch.empty((H, B * L, 2 * S), device=dev, dtype=dt)
    p2c = torch.empty((H, B * L, 2 * S), device=dev, dtype=dt)
    for i in range(cfg.num_hidden_layers):
        p = f"encoder.layer.{i}"
        names = [p + ".attention.self.query_proj", p + ".attention.self.key_proj", p + ".attention.self.value_proj"]
        qkv = Bk.linear_packed(ctx, x, names)                # [B*L, 3D]
        pos = Bk.linear_packed(ctx, relE, names)             # [2S, 3D]: posQ | posK | (unused V)
        for h in range(H):
            qh, kh = qkv[:, h * d:(h + 1) * d], qkv[:, D + h * d:D + (h + 1) * d]
            pqh, pkh = pos[:, h * d:(h + 1) * d], pos[:, D + h * d:D + (h + 1) * d]
            K.gemm(qh, pkh, out=c2p[h])                      # c2p = Q_h posK_h^T  [B*L, 2S]
            K.gemm(kh, pqh, out=p2c[h])                      # p2c = K_h posQ_h^T
        rb = K.deberta_rel_bias(c2p, p2c, c2p_idx, p2c_idx, B, L, scale)
        q3 = qkv.view(B, L, 3 * D)
        o, _ = K.attn_fwd(q3[..., :D], q3[..., D:2 * D], q3[..., 2 * D:], H, scale=scale, key_bias=key_bias,
                          rel_bias=rb)
        K.attn_fill_masked_rows(q3[..., 2 * D:], o, H, mask)
        s1, _ = Bk.linear(ctx, Bk.as2d(o), p + ".attention.output.dense", residual=x)
        h1, _, _ = Bk.layernorm(ctx, s1, p + ".attention.output.LayerNorm", eps)
        f, _ = Bk.linear(ctx, h1, p + ".intermediate.dense", act=K.ACT_GELU)
        s2, _ = Bk.linear(ctx, f, p + ".output.dense", residual=h1)
        x, _, _ = Bk.layernorm(ctx, s2, p + ".output.LayerNorm", eps)
    return x.view(B, L, D)
