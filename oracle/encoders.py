"""TEST INFRASTRUCTURE ONLY (oracle).

CPU restatement of the third-party encoders the reference calls on its hot path
(train.py:137-143 `text_encoder(**inputs).last_hidden_state`, `image_encoder(pixels)
.last_hidden_state`; BASELINE configs use bert-base-uncased and ViT-B/16). The algorithms are
those of transformers 5.15.0 (reference pins 4.47.0, requirements.txt:14; the math of these two
models is unchanged between them):
  BertModel:  BertEmbeddings (word+position+token_type, LayerNorm, dropout), post-LN layers
              (self-attention with the additive extended mask (1-mask)*finfo.min, dense+dropout,
              LayerNorm(x + .), GELU FFN, dense+dropout, LayerNorm(x + .)); no pooler needed for
              last_hidden_state.
  ViTModel:   conv16/s16 patch projection, [CLS] + position embeddings, pre-LN layers
              (layernorm_before -> attention -> + x; layernorm_after -> GELU FFN -> + x), final
              layernorm.
Parameters are dicts with the HF state_dict names. Pinned against transformers' own modules in
tests/golden/make_golden.py.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def _lin(P, n, x):
    return F.linear(x, P[n + ".weight"], P[n + ".bias"])


def _drop(drop, site, x):
    return x if drop is None else drop(site, x)


def _attention(P, pre, h, H, add_mask, drop, site):
    B, L, D = h.shape
    hd = D // H
    q = _lin(P, pre + ".query", h).reshape(B, L, H, hd).transpose(1, 2)
    k = _lin(P, pre + ".key", h).reshape(B, L, H, hd).transpose(1, 2)
    v = _lin(P, pre + ".value", h).reshape(B, L, H, hd).transpose(1, 2)
    s = torch.matmul(q, k.transpose(-1, -2)) / (hd ** 0.5)
    if add_mask is not None:
        s = s + add_mask[:, None, None, :]
    a = torch.softmax(s, dim=-1)
    a = _drop(drop, site + ".attn", a)
    return torch.matmul(a, v).transpose(1, 2).reshape(B, L, D)


def extended_mask(attention_mask, dtype=torch.float32):
    return (1.0 - attention_mask.to(dtype)) * torch.finfo(dtype).min


def bert_forward(P, input_ids, attention_mask=None, token_type_ids=None, *, num_layers, num_heads, eps=1e-12,
                 drop=None, site="bert", pad_token_id=0):
    B, L = input_ids.shape
    if token_type_ids is None:
        token_type_ids = torch.zeros_like(input_ids)
    pos = torch.arange(L)
    # nn.Embedding(vocab, D, padding_idx=pad_token_id): the [PAD] row receives no gradient
    x = (F.embedding(input_ids, P["embeddings.word_embeddings.weight"], padding_idx=pad_token_id)
         + P["embeddings.position_embeddings.weight"][pos][None]
         + P["embeddings.token_type_embeddings.weight"][token_type_ids])
    x = F.layer_norm(x, (x.shape[-1],), P["embeddings.LayerNorm.weight"], P["embeddings.LayerNorm.bias"], eps)
    x = _drop(drop, site + ".emb", x)
    am = extended_mask(attention_mask) if attention_mask is not None else None
    for i in range(num_layers):
        p = f"encoder.layer.{i}"
        s = f"{site}.L{i}"
        ctx = _attention(P, p + ".attention.self", x, num_heads, am, drop, s)
        a = _drop(drop, s + ".attn_out", _lin(P, p + ".attention.output.dense", ctx))
        x = F.layer_norm(a + x, (x.shape[-1],), P[p + ".attention.output.LayerNorm.weight"],
                         P[p + ".attention.output.LayerNorm.bias"], eps)
        f = F.gelu(_lin(P, p + ".intermediate.dense", x))
        o = _drop(drop, s + ".ffn_out", _lin(P, p + ".output.dense", f))
        x = F.layer_norm(o + x, (x.shape[-1],), P[p + ".output.LayerNorm.weight"], P[p + ".output.LayerNorm.bias"], eps)
    return x


def vit_forward(P, pixel_values, *, num_layers, num_heads, patch=16, eps=1e-12, drop=None, site="vit"):
    w = P["embeddings.patch_embeddings.projection.weight"]
    x = F.conv2d(pixel_values, w, P["embeddings.patch_embeddings.projection.bias"], stride=patch)
    x = x.flatten(2).transpose(1, 2)
    B = x.shape[0]
    cls = P["embeddings.cls_token"].expand(B, -1, -1)
    x = torch.cat([cls, x], dim=1) + P["embeddings.position_embeddings"]
    D = x.shape[-1]
    for i in range(num_layers):
        p = f"encoder.layer.{i}"
        s = f"{site}.L{i}"
        h = F.layer_norm(x, (D,), P[p + ".layernorm_before.weight"], P[p + ".layernorm_before.bias"], eps)
        ctx = _attention(P, p + ".attention.attention", h, num_heads, None, drop, s)
        x = _lin(P, p + ".attention.output.dense", ctx) + x
        h = F.layer_norm(x, (D,), P[p + ".layernorm_after.weight"], P[p + ".layernorm_after.bias"], eps)
        x = _lin(P, p + ".output.dense", F.gelu(_lin(P, p + ".intermediate.dense", h))) + x
    return F.layer_norm(x, (D,), P["layernorm.weight"], P["layernorm.bias"], eps)


# ---- MPNet (bi-encoder of the text evidence corpus, text2text_retrieval.py:21,125,129-157) -------
def mpnet_position_ids(input_ids, padding_idx=1):
    """HF create_position_ids_from_input_ids"""
    m = input_ids.ne(padding_idx).int()
    return (torch.cumsum(m, dim=1).type_as(m) * m).long() + padding_idx


def mpnet_buckets(L, num_buckets=32, max_distance=128):
    """HF MPNetEncoder.relative_position_bucket over arange positions"""
    import math
    rel = torch.arange(L)[None, :] - torch.arange(L)[:, None]
    n = -rel
    nb = num_buckets // 2
    ret = (n < 0).long() * nb
    n = n.abs()
    max_exact = nb // 2
    large = max_exact + (torch.log(n.float() / max_exact) / math.log(max_distance / max_exact) * (nb - max_exact)).long()
    large = torch.min(large, torch.full_like(large, nb - 1))
    return ret + torch.where(n < max_exact, n, large)


def mpnet_forward(P, input_ids, attention_mask=None, *, num_layers, num_heads, eps=1e-5, num_buckets=32,
                  padding_idx=1):
    """HF MPNetModel.last_hidden_state (eval): word + position (padding-aware ids) embeddings,
    LayerNorm; post-LN layers whose attention adds the shared relative-position bias and the
    extended mask; GELU FFN."""
    B, L = input_ids.shape
    pos = mpnet_position_ids(input_ids, padding_idx)
    x = F.embedding(input_ids, P["embeddings.word_embeddings.weight"]) + \
        F.embedding(pos, P["embeddings.position_embeddings.weight"])
    D = x.shape[-1]
    x = F.layer_norm(x, (D,), P["embeddings.LayerNorm.weight"], P["embeddings.LayerNorm.bias"], eps)
    bias = F.embedding(mpnet_buckets(L, num_buckets), P["encoder.relative_attention_bias.weight"])  # [L, L, H]
    bias = bias.permute(2, 0, 1)[None]
    add = extended_mask(attention_mask)[:, None, None, :] if attention_mask is not None else 0.0
    H, hd = num_heads, D // num_heads
    for i in range(num_layers):
        p = f"encoder.layer.{i}"
        q = _lin(P, p + ".attention.attn.q", x).reshape(B, L, H, hd).transpose(1, 2)
        k = _lin(P, p + ".attention.attn.k", x).reshape(B, L, H, hd).transpose(1, 2)
        v = _lin(P, p + ".attention.attn.v", x).reshape(B, L, H, hd).transpose(1, 2)
        s = torch.matmul(q, k.transpose(-1, -2)) / (hd ** 0.5) + bias + add
        c = torch.matmul(torch.softmax(s, -1), v).transpose(1, 2).reshape(B, L, D)
        x = F.layer_norm(_lin(P, p + ".attention.attn.o", c) + x, (D,), P[p + ".attention.LayerNorm.weight"],
                         P[p + ".attention.LayerNorm.bias"], eps)
        f = F.gelu(_lin(P, p + ".intermediate.dense", x))
        x = F.layer_norm(_lin(P, p + ".output.dense", f) + x, (D,), P[p + ".output.LayerNorm.weight"],
                         P[p + ".output.LayerNorm.bias"], eps)
    return x


def cross_encoder_forward(P, input_ids, attention_mask, token_type_ids, *, num_layers, num_heads, eps=1e-12,
                          activation="sigmoid"):
    """sentence-transformers 3.3.1 CrossEncoder.predict over HF BertForSequenceClassification
    (num_labels 1), as text2text_retrieval.py:24, 69-79 call it: BERT (keys prefixed "bert."),
    BertPooler tanh(dense(h[:, 0])), classifier Linear -> logits; CrossEncoder's default activation
    for one label is Sigmoid (sentence-transformers is not installed here: its published behaviour
    is restated; `activation=None` returns the raw logits)."""
    B = {k[len("bert."):]: v for k, v in P.items() if k.startswith("bert.")}
    h = bert_forward(B, input_ids, attention_mask, token_type_ids, num_layers=num_layers, num_heads=num_heads,
                     eps=eps)
    pooled = torch.tanh(_lin(P, "bert.pooler.dense", h[:, 0]))
    logits = _lin(P, "classifier", pooled)
    return torch.sigmoid(logits) if activation == "sigmoid" else logits
