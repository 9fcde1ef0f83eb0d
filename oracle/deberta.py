"""TEST INFRASTRUCTURE ONLY (imported by tests/ as the checker; never by the product path).

CPU restatement (plain torch fp32) of the reference's default text encoder, DeBERTa-v3
(`AutoModel.from_pretrained("microsoft/deberta-v3-xsmall")`, train.py:330-331, called at
train.py:136-140, preprocess_embeddings.py:63-80, evaluate.py:112-132). The encoder lives in the
third-party `transformers` package (pinned 4.47.0 at requirements.txt:14; 5.15.0 installed here):
this follows transformers/models/deberta_v2/modeling_deberta_v2.py of the installed version —
make_log_bucket_position / build_relative_position :57-95, DisentangledSelfAttention.forward
:191-274 (scores Q (K / sqrt(3 d)) + c2p + p2c, masked_fill(finfo.min), softmax — a padded query
row therefore averages V over ALL keys), disentangled_attention_bias :276-346 (shared Q/K
projections of the LayerNorm'd relative embeddings, c2p gather at clamp(rel + S), p2c gather at
clamp(-rel + S) transposed), DebertaV2Embeddings.forward :518-560 (word embedding, LayerNorm,
times the mask), the post-LN layer :356-470 and the encoder's rel-embedding LayerNorm :595-600.
Pinned by tests/golden/deberta_small.npz (transformers-built DebertaV2Model; make_golden.py).
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

XSMALL = dict(vocab_size=128100, hidden_size=384, num_hidden_layers=12, num_attention_heads=6,
              intermediate_size=1536, max_position_embeddings=512, position_buckets=256,
              layer_norm_eps=1e-7, pad_token_id=0)


def log_bucket_relative_positions(L: int, bucket_size: int, max_position: int) -> np.ndarray:
    """rel[i, j] = make_log_bucket_position(i - j) (modeling_deberta_v2.py:57-69, 72-95), int64 [L, L]"""
    rel = torch.arange(L)[:, None] - torch.arange(L)[None, :]
    if bucket_size > 0 and max_position > 0:
        sign = torch.sign(rel)
        mid = bucket_size // 2
        abs_pos = torch.where((rel < mid) & (rel > -mid), torch.tensor(mid - 1).type_as(rel), torch.abs(rel))
        log_pos = torch.ceil(torch.log(abs_pos / mid) / torch.log(torch.tensor((max_position - 1) / mid))
                             * (mid - 1)) + mid
        rel = torch.where(abs_pos <= mid, rel.type_as(log_pos), log_pos * sign)
    return rel.to(torch.long).numpy()


def _lin(P, name, x):
    return F.linear(x, P[name + ".weight"], P[name + ".bias"])


def deberta_forward(P, input_ids, attention_mask=None, *, num_layers, num_heads, position_buckets=256,
                    max_position_embeddings=512, eps=1e-7):
    """last_hidden_state [B, L, D] of DebertaV2Model (eval, relative_attention, share_att_key,
    pos_att_type c2p|p2c, norm_rel_ebd layer_norm, position_biased_input False, no token types)."""
    B, L = input_ids.shape
    if attention_mask is None:
        attention_mask = torch.ones_like(input_ids)
    m = attention_mask.to(torch.float32)
    x = F.embedding(input_ids, P["embeddings.word_embeddings.weight"])
    D = x.shape[-1]
    x = F.layer_norm(x, (D,), P["embeddings.LayerNorm.weight"], P["embeddings.LayerNorm.bias"], eps)
    x = x * m[:, :, None]
    ext = attention_mask[:, None, None, :].to(torch.long)
    amask = (ext * ext.squeeze(-2).unsqueeze(-1)).bool()  # [B,1,L,L] = mask[i] * mask[j]
    S = position_buckets if position_buckets > 0 else max_position_embeddings
    rel = torch.from_numpy(log_bucket_relative_positions(L, position_buckets, max_position_embeddings))
    c2p_pos = torch.clamp(rel + S, 0, 2 * S - 1)
    p2c_pos = torch.clamp(-rel + S, 0, 2 * S - 1)
    relE = P["encoder.rel_embeddings.weight"][: 2 * S]
    relE = F.layer_norm(relE, (D,), P["encoder.LayerNorm.weight"], P["encoder.LayerNorm.bias"], eps)
    H = num_heads
    d = D // H
    scale = math.sqrt(d * 3)

    def heads(t):  # [B, L, D] -> [B, H, L, d]
        return t.view(t.shape[0], t.shape[1], H, d).permute(0, 2, 1, 3)

    for i in range(num_layers):
        p = f"encoder.layer.{i}"
        a = p + ".attention.self"
        q = heads(_lin(P, a + ".query_proj", x))
        k = heads(_lin(P, a + ".key_proj", x))
        v = heads(_lin(P, a + ".value_proj", x))
        pq = _lin(P, a + ".query_proj", relE).view(2 * S, H, d).permute(1, 0, 2)  # [H, 2S, d]
        pk = _lin(P, a + ".key_proj", relE).view(2 * S, H, d).permute(1, 0, 2)
        scores = q @ (k / scale).transpose(-1, -2)
        c2p = q @ pk.transpose(-1, -2)                                      # [B,H,L,2S]
        c2p = torch.gather(c2p, -1, c2p_pos.expand(B, H, L, L))
        p2c = k @ pq.transpose(-1, -2)                                      # [B,H,L(key),2S]
        p2c = torch.gather(p2c, -1, p2c_pos.expand(B, H, L, L)).transpose(-1, -2)
        scores = scores + (c2p / scale + p2c / scale)
        scores = scores.masked_fill(~amask, torch.finfo(torch.float32).min)
        ctx = torch.softmax(scores, -1) @ v
        ctx = ctx.permute(0, 2, 1, 3).reshape(B, L, D)
        o = _lin(P, p + ".attention.output.dense", ctx)
        x = F.layer_norm(o + x, (D,), P[p + ".attention.output.LayerNorm.weight"],
                         P[p + ".attention.output.LayerNorm.bias"], eps)
        f = F.gelu(_lin(P, p + ".intermediate.dense", x))
        o = _lin(P, p + ".output.dense", f)
        x = F.layer_norm(o + x, (D,), P[p + ".output.LayerNorm.weight"], P[p + ".output.LayerNorm.bias"], eps)
    return x
