"""TEST INFRASTRUCTURE ONLY (imported by tests/ as the checker; never by the product path).

CPU restatement (plain torch fp32) of the reference's default image encoder, Swinv2
(`Swinv2Model.from_pretrained("microsoft/swinv2-base-patch4-window8-256")`, train.py:332, called at
train.py:142-143 and preprocess_embeddings.py:91-92). The encoder lives in the third-party
`transformers` package (pinned 4.47.0 at requirements.txt:14; 5.15.0 installed here): this follows
transformers/models/swinv2/modeling_swinv2.py of the installed version — window_partition :146-156,
window_reverse :159-167, Swinv2Embeddings.forward :234-260 (patch conv, LayerNorm), PatchMerging
:333-356 (x0 = [0::2, 0::2], x1 = [1::2, 0::2], x2 = [0::2, 1::2], x3 = [1::2, 1::2] -> reduction ->
norm), Swinv2SelfAttention.forward :389-455 (cosine attention times exp(clamp(logit_scale, ln 100)),
16 sigmoid of the continuous position-bias MLP gathered by the relative position index, the shift
mask added twice), create_coords_table_and_index :457-493, Swinv2Layer._compute_window_shift /
get_attn_mask / forward :615-705 (res-post-norm), Swinv2Model.forward :917-985 (final LayerNorm,
AdaptiveAvgPool1d pooler). Pinned by tests/golden/swinv2_small.npz (transformers-built
Swinv2Model; make_golden.py).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

BASE = dict(image_size=256, patch_size=4, num_channels=3, embed_dim=128, depths=(2, 2, 18, 2),
            num_heads=(4, 8, 16, 32), window_size=8, mlp_ratio=4.0, layer_norm_eps=1e-5,
            pretrained_window_sizes=(0, 0, 0, 0))


def _partition(x, ws):
    B, Hh, Ww, C = x.shape
    x = x.view(B, Hh // ws, ws, Ww // ws, ws, C).transpose(2, 3).contiguous()
    return x.view(-1, ws * ws, C)


def _reverse(w, ws, Hh, Ww):
    C = w.shape[-1]
    x = w.view(-1, Hh // ws, Ww // ws, ws, ws, C).transpose(2, 3).contiguous()
    return x.view(-1, Hh, Ww, C)


def _coords(ws, pws):
    r = torch.arange(-(ws - 1), ws).float()
    t = torch.stack(torch.meshgrid([r, r], indexing="ij")).permute(1, 2, 0).contiguous().unsqueeze(0)
    div = (pws - 1) if pws > 0 else (ws - 1 if ws > 1 else None)
    if div is not None:
        t = t / div
    t = t * 8
    t = torch.sign(t) * torch.log2(torch.abs(t) + 1.0) / math.log2(8)
    c = torch.stack(torch.meshgrid([torch.arange(ws), torch.arange(ws)], indexing="ij")).flatten(1)
    rel = (c[:, :, None] - c[:, None, :]).permute(1, 2, 0).contiguous()
    rel[:, :, 0] += ws - 1
    rel[:, :, 1] += ws - 1
    rel[:, :, 0] *= 2 * ws - 1
    return t.reshape(-1, 2), rel.sum(-1)


def _mask(Hh, Ww, ws, shift):
    img = torch.zeros((1, Hh, Ww, 1))
    cnt = 0
    for hs in (slice(0, -ws), slice(-ws, -shift), slice(-shift, None)):
        for wsl in (slice(0, -ws), slice(-ws, -shift), slice(-shift, None)):
            img[:, hs, wsl, :] = cnt
            cnt += 1
    mw = _partition(img, ws).squeeze(-1)
    m = mw.unsqueeze(1) - mw.unsqueeze(2)
    return m.masked_fill(m != 0, -100.0).masked_fill(m == 0, 0.0)


def _attention(sd, p, x, H, ws, mask, pws):
    Bw, L, C = x.shape
    d = C // H
    q = F.linear(x, sd[p + "query.weight"], sd.get(p + "query.bias")).view(Bw, L, H, d).transpose(1, 2)
    k = F.linear(x, sd[p + "key.weight"], sd.get(p + "key.bias")).view(Bw, L, H, d).transpose(1, 2)
    v = F.linear(x, sd[p + "value.weight"], sd.get(p + "value.bias")).view(Bw, L, H, d).transpose(1, 2)
    s = F.normalize(q, dim=-1) @ F.normalize(k, dim=-1).transpose(-2, -1)
    s = s * torch.clamp(sd[p + "logit_scale"], max=math.log(1.0 / 0.01)).exp()
    coords, rpi = _coords(ws, pws)
    hid = F.relu(F.linear(coords, sd[p + "continuous_position_bias_mlp.0.weight"],
                          sd[p + "continuous_position_bias_mlp.0.bias"]))
    table = F.linear(hid, sd[p + "continuous_position_bias_mlp.2.weight"]).view(-1, H)
    rpb = table[rpi.view(-1)].view(L, L, H).permute(2, 0, 1).contiguous()
    s = s + 16 * torch.sigmoid(rpb).unsqueeze(0)
    if mask is not None:
        nW = mask.shape[0]
        s = s.view(Bw // nW, nW, H, L, L) + mask.unsqueeze(1).unsqueeze(0)
        s = s + mask.unsqueeze(1).unsqueeze(0)
        s = s.view(-1, H, L, L)
    a = torch.softmax(s, dim=-1)
    return (a @ v).permute(0, 2, 1, 3).reshape(Bw, L, C)


def _layer(sd, p, x, R, H, window, shift, eps, pws):
    B, N, C = x.shape
    ws = min(R, window)
    if R <= ws:
        shift = 0
    sc = x
    h = x.view(B, R, R, C)
    if shift > 0:
        h = torch.roll(h, shifts=(-shift, -shift), dims=(1, 2))
    w = _partition(h, ws)
    mask = _mask(R, R, ws, shift) if shift > 0 else None
    a = _attention(sd, p + "attention.self.", w, H, ws, mask, pws)
    a = F.linear(a, sd[p + "attention.output.dense.weight"], sd[p + "attention.output.dense.bias"])
    h = _reverse(a.view(-1, ws, ws, C), ws, R, R)
    if shift > 0:
        h = torch.roll(h, shifts=(shift, shift), dims=(1, 2))
    h = h.reshape(B, N, C)
    h = sc + F.layer_norm(h, (C,), sd[p + "layernorm_before.weight"], sd[p + "layernorm_before.bias"], eps)
    f = F.gelu(F.linear(h, sd[p + "intermediate.dense.weight"], sd[p + "intermediate.dense.bias"]))
    f = F.linear(f, sd[p + "output.dense.weight"], sd[p + "output.dense.bias"])
    return h + F.layer_norm(f, (C,), sd[p + "layernorm_after.weight"], sd[p + "layernorm_after.bias"], eps)


def swinv2_forward(sd: dict, pixel_values: torch.Tensor, cfg: dict = BASE):
    """fp32 CPU forward; sd = Swinv2Model state_dict (HF names). Returns (last_hidden_state, pooler_output)."""
    sd = {k: v.detach().float().cpu() for k, v in sd.items()}
    eps = cfg["layer_norm_eps"]
    x = F.conv2d(pixel_values.float().cpu(), sd["embeddings.patch_embeddings.projection.weight"],
                 sd["embeddings.patch_embeddings.projection.bias"], stride=cfg["patch_size"])
    B, C, R, _ = x.shape
    x = x.flatten(2).transpose(1, 2)
    x = F.layer_norm(x, (C,), sd["embeddings.norm.weight"], sd["embeddings.norm.bias"], eps)
    n = len(cfg["depths"])
    for i in range(n):
        H = cfg["num_heads"][i]
        for j in range(cfg["depths"][i]):
            shift = 0 if j % 2 == 0 else cfg["window_size"] // 2
            x = _layer(sd, f"encoder.layers.{i}.blocks.{j}.", x, R, H, cfg["window_size"], shift, eps,
                       cfg["pretrained_window_sizes"][i])
        if i < n - 1:
            Cc = x.shape[-1]
            g = x.view(B, R, R, Cc)
            g = torch.cat([g[:, 0::2, 0::2], g[:, 1::2, 0::2], g[:, 0::2, 1::2], g[:, 1::2, 1::2]], -1)
            g = g.view(B, -1, 4 * Cc)
            p = f"encoder.layers.{i}.downsample."
            g = F.linear(g, sd[p + "reduction.weight"])
            x = F.layer_norm(g, (2 * Cc,), sd[p + "norm.weight"], sd[p + "norm.bias"], eps)
            R //= 2
    x = F.layer_norm(x, (x.shape[-1],), sd["layernorm.weight"], sd["layernorm.bias"], eps)
    return x, x.mean(dim=1)
