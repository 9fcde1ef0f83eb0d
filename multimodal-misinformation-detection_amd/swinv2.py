"""Swinv2 image encoder on HIP kernels — the reference's default image encoder
(`Swinv2Model.from_pretrained("microsoft/swinv2-base-patch4-window8-256")`, train.py:332, called
with `.last_hidden_state` at train.py:142-143 and preprocess_embeddings.py:91-92: [B,3,256,256] ->
[B,64,1024]).

HF parameter names (a hub / transformers state_dict loads unchanged) and HF's arithmetic
(transformers modeling_swinv2.py, restated in oracle/swinv2.py): 4x4 patch conv -> LayerNorm; per
stage `depth` blocks of shifted-window cosine attention with res-post-norm

    h = x + LN_before(W_o . attn(x));   x = h + LN_after(W_2 . gelu(W_1 . h))
    attn: softmax(cos(q_h, k_h) * exp(min(logit_scale_h, ln 100)) + 16 sigmoid(cpb_mlp[rpi]) + 2 mask)

(odd blocks roll the grid by -window/2 first; the mask separates the rolled-in regions and HF adds
it twice), then 2x2 patch merging (concat 4 neighbours -> Linear(4C, 2C, no bias) -> LN); the model
ends in a LayerNorm. Windows never exceed the stage's resolution (window = min(res, 8), no shift
when res <= window).

MI355X mapping: tokens stay `[B*R*R, C]` rows; every block's attention runs over the rows in that
block's (shifted) window order, so the per-token GEMMs / LayerNorms run on the permuted rows as
they are and the only data movement is ONE `mmfd_row_gather` per block that composes the previous
block's order with the next one (roll + window_partition + window_reverse + roll back in a single
pass), and one for each patch merge (which reads the 2x2 neighbours straight out of window order).
QKV is one packed GEMM; the cosine normalisation and the per-head logit scale happen inside the
attention kernel while it stages K and the query fragments (bf16; the fp32 parity mode uses one
in-place pass over the packed rows, `mmfd_swin_qk_norm`); the continuous position bias (+ shift mask) is computed once per block into a
[nW, H, 64, 64] fp32 table that the flash-attention kernel reads with a batch modulus
(`rel_bias_mod`): windows are batch-major per image, so window w of every image shares bias row w.
Inference only (the reference freezes its encoders, train.py:335-340, and the pre-embedding pass
runs under no_grad): a forward that would need gradients raises.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np
import torch
import torch.nn as nn

from . import blocks as Bk
from . import kernels as K
from .encoders import EncoderOutput


@dataclass
class Swinv2Config:
    """microsoft/swinv2-base-patch4-window8-256 defaults"""
    image_size: int = 256
    patch_size: int = 4
    num_channels: int = 3
    embed_dim: int = 128
    depths: tuple = (2, 2, 18, 2)
    num_heads: tuple = (4, 8, 16, 32)
    window_size: int = 8
    mlp_ratio: float = 4.0
    qkv_bias: bool = True
    layer_norm_eps: float = 1e-5
    pretrained_window_sizes: tuple = (0, 0, 0, 0)


# ------------------------------------------------------------------------------------------------
# host-side geometry (constants per (resolution, window, shift); cached on the device)
# ------------------------------------------------------------------------------------------------
def stage_geometry(cfg: Swinv2Config):
    """[(R, dim, heads, [(window, shift) per block])] per stage (Swinv2Encoder / Swinv2Layer
    _compute_window_shift)"""
    R = cfg.image_size // cfg.patch_size
    out = []
    for i, depth in enumerate(cfg.depths):
        Ri = R // (2 ** i)
        ws = min(Ri, cfg.window_size)
        blocks = []
        for j in range(depth):
            shift = 0 if (j % 2 == 0) else cfg.window_size // 2
            if Ri <= ws:
                shift = 0
            blocks.append((ws, shift))
        out.append((Ri, int(cfg.embed_dim * 2 ** i), cfg.num_heads[i], blocks))
    return out


def window_order(R, ws, shift):
    """natural raster index of every row in (rolled by -shift) window order: window (wy, wx)
    batch-major, tokens row-major inside the window (torch.roll + window_partition)"""
    n = R // ws
    wy, wx, iy, ix = np.meshgrid(np.arange(n), np.arange(n), np.arange(ws), np.arange(ws), indexing="ij")
    y = (wy * ws + iy + shift) % R
    x = (wx * ws + ix + shift) % R
    return (y * R + x).reshape(-1).astype(np.int64)


def shift_mask(R, ws, shift):
    """[nW, L, L] fp32: 0 within a cyclic-shift region, -100 across (Swinv2Layer.get_attn_mask)"""
    idx = np.arange(R)
    reg = (idx >= R - ws).astype(np.int64) + (idx >= R - shift).astype(np.int64)
    img = reg[:, None] * 3 + reg[None, :]                         # label on the rolled grid
    n = R // ws
    lab = img.reshape(n, ws, n, ws).transpose(0, 2, 1, 3).reshape(n * n, ws * ws)
    m = lab[:, None, :] - lab[:, :, None]
    return np.where(m != 0, -100.0, 0.0).astype(np.float32)


def coords_table_and_index(ws, pretrained_ws=0):
    """(relative_coords_table [(2ws-1)^2, 2] fp32, relative_position_index int32 [ws^2 * ws^2])
    as Swinv2SelfAttention.create_coords_table_and_index (computed with torch on the host)"""
    rh = torch.arange(-(ws - 1), ws, dtype=torch.int64).float()
    t = torch.stack(torch.meshgrid([rh, rh], indexing="ij")).permute(1, 2, 0).contiguous().unsqueeze(0)
    if pretrained_ws > 0:
        t[:, :, :, 0] /= pretrained_ws - 1
        t[:, :, :, 1] /= pretrained_ws - 1
    elif ws > 1:
        t[:, :, :, 0] /= ws - 1
        t[:, :, :, 1] /= ws - 1
    t *= 8
    t = torch.sign(t) * torch.log2(torch.abs(t) + 1.0) / math.log2(8)
    c = torch.stack(torch.meshgrid([torch.arange(ws), torch.arange(ws)], indexing="ij")).flatten(1)
    rel = (c[:, :, None] - c[:, None, :]).permute(1, 2, 0).contiguous()
    rel[:, :, 0] += ws - 1
    rel[:, :, 1] += ws - 1
    rel[:, :, 0] *= 2 * ws - 1
    return t.reshape(-1, 2).float(), rel.sum(-1).reshape(-1).to(torch.int32)


class _Geo:
    """device-resident index tables / masks, built once per (device, config)"""

    def __init__(self, dev):
        self.dev = dev
        self._c = {}

    def get(self, key, make):
        t = self._c.get(key)
        if t is None:
            t = self._c[key] = make()
        return t

    def idx(self, arr):
        return torch.from_numpy(np.ascontiguousarray(arr, dtype=np.int32)).to(self.dev)


# ------------------------------------------------------------------------------------------------
# module tree (HF names)
# ------------------------------------------------------------------------------------------------
def _linear(i, o, bias=True):
    return nn.Linear(i, o, bias=bias)


class Swinv2Model(Bk.CachedWeights, nn.Module):
    def __init__(self, config: Swinv2Config | None = None, **kw):
        super().__init__()
        c = config or Swinv2Config(**kw)
        self.config = c
        eps = c.layer_norm_eps
        self.embeddings = nn.Module()
        self.embeddings.patch_embeddings = nn.Module()
        self.embeddings.patch_embeddings.projection = nn.Conv2d(c.num_channels, c.embed_dim, c.patch_size,
                                                                stride=c.patch_size)
        self.embeddings.norm = nn.LayerNorm(c.embed_dim, eps=eps)
        self.encoder = nn.Module()
        self.encoder.layers = nn.ModuleList()
        geo = stage_geometry(c)
        for i, (R, dim, H, blocks) in enumerate(geo):
            st = nn.Module()
            st.blocks = nn.ModuleList()
            for _ in blocks:
                b = nn.Module()
                b.attention = nn.Module()
                s = b.attention.self = nn.Module()
                s.logit_scale = nn.Parameter(torch.log(10 * torch.ones((H, 1, 1))))
                s.continuous_position_bias_mlp = nn.Sequential(nn.Linear(2, 512, bias=True), nn.ReLU(inplace=True),
                                                               nn.Linear(512, H, bias=False))
                s.query = _linear(dim, dim, c.qkv_bias)
                s.key = _linear(dim, dim, False)
                s.value = _linear(dim, dim, c.qkv_bias)
                b.attention.output = nn.Module()
                b.attention.output.dense = _linear(dim, dim)
                b.layernorm_before = nn.LayerNorm(dim, eps=eps)
                b.intermediate = nn.Module()
                b.intermediate.dense = _linear(dim, int(c.mlp_ratio * dim))
                b.output = nn.Module()
                b.output.dense = _linear(int(c.mlp_ratio * dim), dim)
                b.layernorm_after = nn.LayerNorm(dim, eps=eps)
                st.blocks.append(b)
            if i < len(geo) - 1:
                st.downsample = nn.Module()
                st.downsample.reduction = _linear(4 * dim, 2 * dim, False)
                st.downsample.norm = nn.LayerNorm(2 * dim, eps=eps)
            self.encoder.layers.append(st)
        nf = int(c.embed_dim * 2 ** (len(c.depths) - 1))
        self.layernorm = nn.LayerNorm(nf, eps=eps)
        self.num_features = nf
        self.compute_dtype = torch.float32
        self._geo = {}
        self._init_weights()

    def _init_weights(self, std=0.02):
        """Swinv2PreTrainedModel._init_weights: normal(0, 0.02) Linear/Conv, zero bias, LN 1/0"""
        for m in self.modules():
            if isinstance(m, (nn.Linear, nn.Conv2d)):
                nn.init.normal_(m.weight, 0.0, std)
                if m.bias is not None:
                    nn.init.zeros_(m.bias)
            elif isinstance(m, nn.LayerNorm):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)

    def set_precision(self, precision):
        self.compute_dtype = {"fp32": torch.float32, "bf16": torch.bfloat16}[precision]
        return self

    def forward(self, pixel_values, **unused):
        params = dict(self.named_parameters())
        first = next(iter(params.values()))
        if not first.is_cuda:
            raise RuntimeError("mmfd Swinv2Model runs on the HIP device: call .to('cuda') first")
        if torch.is_grad_enabled() and any(p.requires_grad for p in params.values()):
            raise NotImplementedError("mmfd Swinv2Model is inference-only (frozen encoder, train.py:335-340): "
                                      "call it under torch.no_grad() or freeze its parameters")
        P = {n: p.detach() for n, p in params.items()}
        pw = "embeddings.patch_embeddings.projection.weight"
        P[pw] = P[pw].reshape(P[pw].shape[0], -1)               # conv as a [C_out, 3*p*p] GEMM weight
        ctx = Bk.StepCtx(P, self.compute_dtype, shadows=Bk.shadow_store(self))
        ctx.cache_derived = True          # frozen encoder: packed biases / position-bias tables persist
        geo = self._geo.get(str(first.device))
        if geo is None:
            geo = self._geo[str(first.device)] = _Geo(first.device)
        out = swinv2_forward(self, ctx, geo, pixel_values)
        pooled = K.seq_mean_fwd(out)                               # Swinv2Model.pooler (AdaptiveAvgPool1d)
        return EncoderOutput(last_hidden_state=out, extra={"pooler_output": pooled})


def swinv2_forward(model: Swinv2Model, ctx: Bk.StepCtx, geo: _Geo, pixel_values):
    cfg = model.config
    dev = ctx.P["layernorm.weight"].device
    px = pixel_values.to(dev)
    B, Cin, Hh, Ww = px.shape
    p = cfg.patch_size
    if Hh != cfg.image_size or Ww != cfg.image_size or Cin != cfg.num_channels:
        raise ValueError(f"Swinv2Model expects [B,{cfg.num_channels},{cfg.image_size},{cfg.image_size}] pixels, "
                         f"got {tuple(px.shape)}")
    eps = cfg.layer_norm_eps
    dt = ctx.dt
    # embeddings: conv 4x4/4 as patchify + GEMM, then LayerNorm (dropout is identity in eval)
    x = K.patchify(px.float().contiguous(), p, dt)              # [B*R*R, 3*p*p]
    x, _ = Bk.linear(ctx, x, "embeddings.patch_embeddings.projection")
    x, _, _ = Bk.layernorm(ctx, x, "embeddings.norm", eps)
    stages = stage_geometry(cfg)
    for i, (R, dim, H, blocks) in enumerate(stages):
        d = dim // H
        order = np.arange(R * R)                                # natural index of each row
        inv = np.arange(R * R)
        for j, (ws, shift) in enumerate(blocks):
            pre = f"encoder.layers.{i}.blocks.{j}"
            L = ws * ws
            nW = (R // ws) ** 2
            tgt = window_order(R, ws, shift)
            if not np.array_equal(tgt, order):
                idx = geo.get(("perm", i, j), lambda: geo.idx(inv[tgt]))
                x = K.row_gather(x, idx, B, R * R)
                order = tgt
                inv = np.empty_like(order)
                inv[order] = np.arange(R * R)
            x = _swin_block(ctx, geo, x, pre, B, R, dim, H, d, ws, shift, nW, L, eps, cfg)
        if i < len(stages) - 1:
            # patch merging: out (y2, x2) = [x(2y2,2x2), x(2y2+1,2x2), x(2y2,2x2+1), x(2y2+1,2x2+1)]
            R2 = R // 2
            y2, x2 = np.meshgrid(np.arange(R2), np.arange(R2), indexing="ij")
            y2, x2 = y2.reshape(-1), x2.reshape(-1)
            nat = np.stack([(2 * y2) * R + 2 * x2, (2 * y2 + 1) * R + 2 * x2, (2 * y2) * R + 2 * x2 + 1,
                            (2 * y2 + 1) * R + 2 * x2 + 1], axis=1).reshape(-1)
            idx = geo.get(("merge", i), lambda: geo.idx(inv[nat]))
            xm = K.row_gather(x, idx, B, R2 * R2, G=4)            # [B*R2*R2, 4*dim]
            pre = f"encoder.layers.{i}.downsample"
            x, _ = Bk.linear(ctx, xm, pre + ".reduction")
            x, _, _ = Bk.layernorm(ctx, x, pre + ".norm", eps)
        elif not np.array_equal(order, np.arange(R * R)):
            idx = geo.get(("final", i), lambda: geo.idx(inv[np.arange(R * R)]))
            x = K.row_gather(x, idx, B, R * R)
    x, _, _ = Bk.layernorm(ctx, x, "layernorm", eps)
    Rl = stages[-1][0]
    return x.view(B, Rl * Rl, -1)


def _swin_block(ctx, geo, x, pre, B, R, dim, H, d, ws, shift, nW, L, eps, cfg):
    s = pre + ".attention.self"
    qkv = Bk.linear_packed(ctx, x, [s + ".query", s + ".key", s + ".value"])   # [N, 3*dim]
    fused = ctx.dt == torch.bfloat16          # bf16: the attention kernel normalises q / k while staging
    if not fused:
        K.swin_qk_norm(qkv, H, d, ctx.P[s + ".logit_scale"], math.log(1.0 / 0.01))
    stage = int(pre.split(".")[2])
    pws = cfg.pretrained_window_sizes[stage]
    coords, rpi = geo.get(("cpb", ws, pws), lambda: tuple(t.to(geo.dev) for t in coords_table_and_index(ws, pws)))
    cpb = [s + ".continuous_position_bias_mlp.0.weight", s + ".continuous_position_bias_mlp.0.bias",
           s + ".continuous_position_bias_mlp.2.weight"]
    mask = None
    if shift > 0:
        mask = geo.get(("mask", R, ws, shift), lambda: torch.from_numpy(shift_mask(R, ws, shift)).to(geo.dev))
    # [nW|1, H, L, L]: depends on the block's weights only -> rebuilt only when they change
    bias = ctx.derived(s + "#swin_bias", cpb,
                       lambda: K.swin_bias(K.swin_cpb(coords, *[ctx.P[n] for n in cpb]), rpi, L, mask))
    q3 = qkv.view(B * nW, L, 3 * dim)
    o, _ = K.attn_fwd(q3[..., :dim], q3[..., dim:2 * dim], q3[..., 2 * dim:], H, scale=1.0,
                      rel_bias=bias if shift > 0 else bias.view(H, L, L),
                      cos_logit_scale=ctx.P[s + ".logit_scale"].view(-1) if fused else None,
                      cos_max_log=math.log(1.0 / 0.01))
    y, _ = Bk.linear(ctx, Bk.as2d(o), pre + ".attention.output.dense")
    h = K.layernorm_fwd_res(y, ctx.P[pre + ".layernorm_before.weight"], ctx.P[pre + ".layernorm_before.bias"], eps,
                            res=x)
    f, _ = Bk.linear(ctx, h, pre + ".intermediate.dense", act=K.ACT_GELU)
    m, _ = Bk.linear(ctx, f, pre + ".output.dense")
    return K.layernorm_fwd_res(m, ctx.P[pre + ".layernorm_after.weight"], ctx.P[pre + ".layernorm_after.bias"], eps,
                               res=h)
