"""Swinv2 image encoder (the reference's default, train.py:332) on the HIP path vs the transformers
fixture (tests/golden/swinv2_small.npz: shifted windows with 16 and 4 windows per image, a single
8x8 window, a logit scale above the clamp) and vs the CPU oracle (oracle/swinv2.py) at the
swinv2-base-patch4-window8-256 shape; plus the Swin-specific kernels one by one.
Tolerances: fp32 1e-4 abs vs the fixture, 1e-3 abs at the base shape (north_star's logit bar);
bf16 0.25 max abs on the 24-block LayerNorm'd outputs (the bar of the other full-size bf16 encoder
tests) plus 2e-2 mean abs, which a wrong permutation, bias row or mask would exceed."""
import math
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
SMALL = dict(image_size=128, embed_dim=32, depths=(2, 2, 2), num_heads=(1, 2, 4), pretrained_window_sizes=(0, 0, 0))


def test_row_gather_windows_and_merge():
    from mmfd import kernels as K
    from mmfd.swinv2 import window_order
    B, R, C = 3, 16, 40
    x = torch.randn(B * R * R, C, device="cuda")
    order = window_order(R, 8, 4)
    idx = torch.from_numpy(order.astype(np.int32)).cuda()
    y = K.row_gather(x, idx, B, R * R)
    want = x.view(B, R * R, C)[:, torch.from_numpy(order).cuda()].reshape(B * R * R, C)
    assert torch.equal(y, want)
    nat = torch.arange(R * R).view(R, R)
    four = torch.stack([nat[0::2, 0::2], nat[1::2, 0::2], nat[0::2, 1::2], nat[1::2, 1::2]], -1).reshape(-1)
    m = K.row_gather(x.bfloat16(), four.int().cuda(), B, (R // 2) ** 2, G=4)
    xb = x.bfloat16().view(B, R, R, C)
    wantm = torch.cat([xb[:, 0::2, 0::2], xb[:, 1::2, 0::2], xb[:, 0::2, 1::2], xb[:, 1::2, 1::2]], -1)
    assert torch.equal(m, wantm.reshape(-1, 4 * C))


@pytest.mark.parametrize("H,shift", [(4, 0), (4, 4), (32, 0)])
def test_swin_bias_and_cpb(H, shift):
    from mmfd import kernels as K
    from mmfd.swinv2 import coords_table_and_index, shift_mask
    ws, R = 8, 32
    coords, rpi = coords_table_and_index(ws)
    torch.manual_seed(H)
    w1, b1, w2 = torch.randn(512, 2) * 0.5, torch.randn(512) * 0.1, torch.randn(H, 512) * 0.05
    table = K.swin_cpb(coords.cuda(), w1.cuda(), b1.cuda(), w2.cuda())
    want_t = torch.relu(coords @ w1.T + b1) @ w2.T
    assert (table.cpu() - want_t).abs().max().item() < 1e-4
    mask = torch.from_numpy(shift_mask(R, ws, shift)).cuda() if shift else None
    bias = K.swin_bias(table, rpi.cuda(), ws * ws, mask)
    want = 16 * torch.sigmoid(table.cpu()[rpi.long()].view(64, 64, H).permute(2, 0, 1)).unsqueeze(0)
    if shift:
        m = mask.cpu().unsqueeze(1)
        want = (want + m) + m
    assert bias.shape == want.shape
    err = ((bias.cpu() - want).abs() / (1 + want.abs())).max().item()
    assert err < 1e-6, err


@pytest.mark.parametrize("dt,d", [(torch.float32, 32), (torch.bfloat16, 32), (torch.float32, 64)])
def test_swin_qk_norm(dt, d):
    from mmfd import kernels as K
    H, rows = 4, 300
    qkv = torch.randn(rows, 3 * H * d, device="cuda").to(dt)
    qkv[5, :d] = 0  # all-zero head: F.normalize's eps path
    ls = torch.tensor([0.5, 2.3, 5.0, -1.0], device="cuda")
    ref = qkv.float().view(rows, 3, H, d).clone()
    out = K.swin_qk_norm(qkv.clone(), H, d, ls, math.log(100.0)).float().view(rows, 3, H, d)
    sc = torch.clamp(ls, max=math.log(100.0)).exp().view(1, H, 1)
    wq = torch.nn.functional.normalize(ref[:, 0], dim=-1) * sc
    wk = torch.nn.functional.normalize(ref[:, 1], dim=-1)
    tol = 1e-5 if dt == torch.float32 else 4e-2
    assert (out[:, 0] - wq).abs().max().item() < tol * 100
    assert (out[:, 1] - wk).abs().max().item() < tol
    assert torch.equal(out[:, 2], ref[:, 2])


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_layernorm_fwd_res(dt):
    from mmfd import kernels as K
    x = torch.randn(517, 1024, device="cuda").to(dt)
    r = torch.randn(517, 1024, device="cuda").to(dt)
    g, b = torch.randn(1024, device="cuda"), torch.randn(1024, device="cuda")
    y = K.layernorm_fwd_res(x, g, b, 1e-5, res=r)
    want = r.float() + torch.nn.functional.layer_norm(x.float(), (1024,), g, b, 1e-5)
    assert (y.float() - want).abs().max().item() < (1e-4 if dt == torch.float32 else 6e-2)


def test_attention_bias_modulus_matches_per_window_bias():
    """rel_bias [nW, H, L, L] read with batch modulus == the same bias tiled to [B*nW, H, L, L]"""
    from mmfd import kernels as K
    Bi, nW, H, L, D = 3, 4, 2, 64, 32
    q = torch.randn(Bi * nW, L, H * D, device="cuda")
    k = torch.randn(Bi * nW, L, H * D, device="cuda")
    v = torch.randn(Bi * nW, L, H * D, device="cuda")
    bias = torch.randn(nW, H, L, L, device="cuda")
    bias[1, :, :, 7] = -200.0
    o1, _ = K.attn_fwd(q, k, v, H, scale=0.3, rel_bias=bias)
    o2, _ = K.attn_fwd(q, k, v, H, scale=0.3, rel_bias=bias.repeat(Bi, 1, 1, 1).contiguous())
    torch.cuda.synchronize()
    assert torch.equal(o1, o2)


@pytest.mark.parametrize("nW,L", [(4, 64), (1, 64), (2, 16)])
def test_attention_fused_cosine_matches_separate_pass(nW, L):
    """bf16 attention with cos_logit_scale (q/k normalised while staged) == mmfd_swin_qk_norm followed
    by plain attention, on the same bf16 inputs"""
    from mmfd import kernels as K
    Bi, H, d = 3, 4, 32
    torch.manual_seed(L + nW)
    qkv = (torch.randn(Bi * nW * L, 3 * H * d, device="cuda") * 2).bfloat16()
    qkv[7, :d] = 0
    ls = torch.tensor([0.5, 2.3, 5.0, -1.0], device="cuda")
    bias = torch.randn(nW, H, L, L, device="cuda")
    sep = K.swin_qk_norm(qkv.clone(), H, d, ls, math.log(100.0)).view(Bi * nW, L, 3 * H * d)
    o1, _ = K.attn_fwd(sep[..., :H * d], sep[..., H * d:2 * H * d], sep[..., 2 * H * d:], H, scale=1.0, rel_bias=bias)
    q3 = qkv.view(Bi * nW, L, 3 * H * d)
    o2, _ = K.attn_fwd(q3[..., :H * d], q3[..., H * d:2 * H * d], q3[..., 2 * H * d:], H, scale=1.0, rel_bias=bias,
                       cos_logit_scale=ls, cos_max_log=math.log(100.0))
    torch.cuda.synchronize()
    assert (o1.float() - o2.float()).abs().max().item() < 2e-2


def _cfg(**kw):
    from mmfd.swinv2 import Swinv2Config
    return Swinv2Config(**kw)


def test_swinv2_matches_transformers_fixture():
    from mmfd.swinv2 import Swinv2Model
    z = np.load(os.path.join(G, "swinv2_small.npz"))
    m = Swinv2Model(_cfg(**SMALL))
    m.load_state_dict({k[2:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("w.")})
    m = m.cuda().eval()
    with torch.no_grad():
        o = m(torch.from_numpy(z["pixel_values"]).cuda())
    torch.cuda.synchronize()
    err = (o.last_hidden_state.cpu() - torch.from_numpy(z["last_hidden_state"])).abs().max().item()
    assert err < 1e-4, err
    perr = (o.extra["pooler_output"].cpu() - torch.from_numpy(z["pooler_output"])).abs().max().item()
    assert perr < 1e-4, perr


@pytest.mark.parametrize("precision,tol", [("fp32", 1e-3), ("bf16", 0.25)])
def test_swinv2_base_vs_oracle(precision, tol):
    """swinv2-base-patch4-window8-256 shape (embed 128, depths 2/2/18/2, heads 4/8/16/32, window 8):
    [2,3,256,256] -> [2,64,1024], random init moved off the trivial LayerNorm / bias values"""
    from mmfd.swinv2 import Swinv2Model
    from oracle.swinv2 import swinv2_forward
    torch.manual_seed(5)
    m = Swinv2Model()
    with torch.no_grad():
        for q in m.parameters():
            q.add_(torch.randn_like(q) * 0.02)
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    m = m.cuda().eval().set_precision(precision)
    px = torch.randn(2, 3, 256, 256, generator=torch.Generator().manual_seed(6))
    with torch.no_grad():
        out = m(px.cuda()).last_hidden_state
        want, _ = swinv2_forward(sd, px)
    torch.cuda.synchronize()
    assert tuple(out.shape) == (2, 64, 1024)
    d = (out.float().cpu() - want).abs()
    assert d.max().item() < tol, d.max().item()
    if precision == "bf16":
        assert d.mean().item() < 2e-2, d.mean().item()


def test_swinv2_refuses_grad_and_cpu():
    from mmfd.swinv2 import Swinv2Model
    m = Swinv2Model(_cfg(**SMALL))
    with pytest.raises(RuntimeError):
        m(torch.zeros(1, 3, 128, 128))
    m = m.cuda()
    with pytest.raises(NotImplementedError):
        m(torch.zeros(1, 3, 128, 128, device="cuda"))


def test_swinv2_weight_change_rebuilds_cached_bias():
    """the per-block position-bias tables and packed QKV biases persist across calls (frozen
    encoder) and are rebuilt when a weight changes in place"""
    from mmfd.swinv2 import Swinv2Model
    from oracle.swinv2 import swinv2_forward
    z = np.load(os.path.join(G, "swinv2_small.npz"))
    m = Swinv2Model(_cfg(**SMALL))
    m.load_state_dict({k[2:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("w.")})
    m = m.cuda().eval()
    px = torch.from_numpy(z["pixel_values"])
    with torch.no_grad():
        a = m(px.cuda()).last_hidden_state.clone()
        b = m(px.cuda()).last_hidden_state
        assert torch.equal(a, b)
        blk = m.encoder.layers[0].blocks[1].attention.self
        blk.continuous_position_bias_mlp[2].weight.mul_(3.0)
        blk.query.bias.add_(0.5)
        c = m(px.cuda()).last_hidden_state
        want, _ = swinv2_forward({k: v.cpu() for k, v in m.state_dict().items()}, px, dict(
            image_size=128, patch_size=4, num_channels=3, embed_dim=32, depths=(2, 2, 2), num_heads=(1, 2, 4),
            window_size=8, mlp_ratio=4.0, layer_norm_eps=1e-5, pretrained_window_sizes=(0, 0, 0)))
    torch.cuda.synchronize()
    assert (c.cpu() - want).abs().max().item() < 1e-4
    assert (c - a).abs().max().item() > 1e-3
