"""Fusion head (MisinformationDetectionModel) on the HIP path vs the reference fixtures and the
pinned CPU oracle.

Tolerances: fp32 mode — logits/losses 1e-4 abs (north_star: within 1e-3), parameter gradients
2e-4 relative to the tensor's max; bf16 mode — logits 5e-2 abs (bf16 operands, fp32 accumulate).
"""
import json
import os

import numpy as np
import pytest
import torch

import mmfd
from mmfd import kernels as K
from mmfd.model import MisinformationDetectionModel
from mmfd.optim import AdamW
from oracle import fusion_head as OF
from oracle.dropout_hash import make_drop

pytestmark = pytest.mark.gpu
DEV = "cuda"
G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
SMALL = dict(text_input_dim=48, image_input_dim=40, embed_dim=32, num_heads=4, hidden_dim=16)


def _z(name):
    return np.load(os.path.join(G, name), allow_pickle=False)


def _t(a, dev=DEV):
    return torch.from_numpy(np.array(a)).to(dev)


def _close(got, ref, tol):
    got = torch.as_tensor(got).detach().double().cpu()
    ref = torch.as_tensor(np.asarray(ref) if not torch.is_tensor(ref) else ref).detach().double().cpu()
    assert got.shape == ref.shape
    err = (got - ref).abs().max().item()
    assert err <= tol, f"max abs err {err:.3e} > {tol:.1e}"
    return err


def _model(z, prefix="init/", dropout=0.0, **kw):
    m = MisinformationDetectionModel(**{**SMALL, **kw}, dropout=dropout)
    m.load_state_dict({k[len(prefix):]: torch.from_numpy(z[k]) for k in z.files if k.startswith(prefix)})
    return m.to(DEV)


def test_eval_modes_match_reference():
    z = _z("fusion_small.npz")
    X = [_t(z[k]) for k in ("X_t", "X_i", "E_t", "E_i")]
    m = _model(z).eval()
    with torch.no_grad():
        (a, b), (c, d) = m(*X)
        for y, k in zip((a, b, c, d), ("tt", "ti", "it", "ii")):
            _close(y, z[f"eval_{k}"], 1e-4)
        (u, n1), (n2, n3) = m(X_t=X[0], E_t=X[2])
        assert n1 is None and n2 is None and n3 is None
        _close(u, z["uni_tt"], 1e-4)
        mf = _model(z, "factify_init/", factify=True, num_classes=5).eval()
        y, none = mf(*X)
        assert none is None
        _close(y, z["factify_out"], 1e-4)
        mt = _model(z, "text_only_init/", text_only=True).eval()
        y, _ = mt(X_t=X[0], E_t=X[2])
        _close(y, z["text_only_out"], 1e-4)


def test_train_step_matches_reference_train_epoch():
    """train.py:123-188 with the reference's own fixture: zero_grad, forward, 4x CE, backward, AdamW."""
    z = _z("fusion_small.npz")
    X = [_t(z[k]) for k in ("X_t", "X_i", "E_t", "E_i")]
    labels = _t(z["labels"])
    m = _model(z).train()
    opt = AdamW(m.parameters(), lr=1e-4)
    opt.zero_grad()
    (a, b), (c, d) = m(*X)
    crit = torch.nn.CrossEntropyLoss()
    losses = [crit(y, labels[:, i]) for i, y in enumerate((a, b, c, d))]
    total = sum(losses)
    _close(total, z["train_total_loss"], 1e-4)
    for l, n in zip(losses, ("text_text", "text_image", "image_text", "image_image")):
        _close(l, z[f"train_loss_{n}"], 1e-4)
    total.backward()
    names = [k for k, _ in json.loads(str(z["param_names"]))]
    P = dict(m.named_parameters())
    for k in names:
        if "grad/" + k in z.files:
            ref = z["grad/" + k]
            _close(P[k].grad, ref, 2e-4 * max(1.0, np.abs(ref).max()))
        else:
            assert P[k].grad is None, k
    opt.step()
    # AdamW's first step moves each element by ~lr * g / (|g| + eps): an element whose reference
    # gradient is within fp32 noise of 0 (|g| < 1e-6) moves by up to lr in the direction of that
    # noise's sign, so the two steps may differ by up to 2 lr there; all others must agree
    for k in names:
        post = P[k].detach().double().cpu()
        ref = torch.from_numpy(z["post/" + k]).double()
        diff = (post - ref).abs()
        assert diff.max().item() <= 2.0001e-4 + 1e-6, k
        if "grad/" + k in z.files:
            solid = torch.from_numpy(z["grad/" + k]).abs() > 1e-6
            worst = diff[solid].max().item() if solid.any() else 0.0
            assert worst <= 2e-6, (k, worst)
    # the optimizer alone, fed the reference gradients, reproduces the reference step exactly
    m2 = _model(z)
    opt2 = AdamW(m2.parameters(), lr=1e-4)
    for k, p in m2.named_parameters():
        p.grad = _t(z["grad/" + k]) if "grad/" + k in z.files else None
    opt2.step()
    for k, p in m2.named_parameters():
        _close(p, z["post/" + k], 1e-7)


def test_xent_kernel_in_train_step():
    z = _z("fusion_small.npz")
    X = [_t(z[k]) for k in ("X_t", "X_i", "E_t", "E_i")]
    m = _model(z).train()
    (a, b), (c, d) = m(*X)
    loss, dl = K.xent_fwd_bwd([a.detach(), b.detach(), c.detach(), d.detach()], _t(z["labels"]))
    _close(loss[0], z["train_total_loss"], 1e-4)


@pytest.mark.parametrize("factify,text_only", [(False, False), (True, False), (False, True)])
def test_train_mode_dropout_matches_oracle(factify, text_only):
    """Train mode, dropout 0.1 everywhere: identical counter-based masks in the oracle."""
    z = _z("fusion_small.npz")
    g = torch.Generator().manual_seed(5)
    B, shapes = 3, dict(X_t=(3, 10, 48), X_i=(3, 17, 40), E_t=(3, 12, 48), E_i=(3, 9, 40))
    Xc = {k: torch.randn(*s, generator=g) for k, s in shapes.items()}
    kw = dict(factify=factify, num_classes=5 if factify else 3, text_only=text_only)
    m = MisinformationDetectionModel(**SMALL, dropout=0.1, **kw).to(DEV).train()
    m.manual_seed(4242)
    P = {n: p.detach().cpu().clone().requires_grad_(True) for n, p in m.named_parameters()}
    Xg = {k: v.to(DEV).requires_grad_(True) for k, v in Xc.items()}
    Xr = {k: v.clone().requires_grad_(True) for k, v in Xc.items()}
    drop = make_drop(4242, 0.1)
    if text_only:
        y, _ = m(X_t=Xg["X_t"], E_t=Xg["E_t"])
        yr, _ = OF.model_forward(P, X_t=Xr["X_t"], E_t=Xr["E_t"], num_heads=4, text_only=True, drop=drop)
        ys, yrs = [y], [yr]
    elif factify:
        y, _ = m(*Xg.values())
        yr, _ = OF.model_forward(P, *Xr.values(), num_heads=4, factify=True, drop=drop)
        ys, yrs = [y], [yr]
    else:
        (a, b), (c, d) = m(*Xg.values())
        (ar, br), (cr, dr) = OF.model_forward(P, *Xr.values(), num_heads=4, drop=drop)
        ys, yrs = [a, b, c, d], [ar, br, cr, dr]
    Rs = [torch.randn(y.shape, generator=g) for y in ys]
    for y, yr in zip(ys, yrs):
        _close(y, yr, 1e-4)
    sum((y * R.to(DEV)).sum() for y, R in zip(ys, Rs)).backward()
    sum((y * R).sum() for y, R in zip(yrs, Rs)).backward()
    for n, p in m.named_parameters():
        if P[n].grad is None:
            assert p.grad is None, n
            continue
        ref = P[n].grad
        _close(p.grad, ref, 3e-4 * max(1.0, ref.abs().max().item()))
    for k in Xg:
        if Xr[k].grad is not None:
            _close(Xg[k].grad, Xr[k].grad, 3e-4 * max(1.0, Xr[k].grad.abs().max().item()))


def test_full_dims_logits_fp32_and_bf16():
    z = _z("fusion_full.npz")
    names = json.loads(str(z["param_names"]))
    P = OF.init_params_like_reference(names, int(z["seed"]))
    m = MisinformationDetectionModel(text_input_dim=768, image_input_dim=768)
    m.load_state_dict(P)
    m = m.to(DEV).eval()
    X = [_t(z[k]) for k in ("X_t", "X_i", "E_t", "E_i")]
    with torch.no_grad():
        (a, b), (c, d) = m(*X)
        for y, k in zip((a, b, c, d), ("tt", "ti", "it", "ii")):
            _close(y, z[k], 1e-4)
        m.set_precision("bf16")
        (a, b), (c, d) = m(*X)
        for y, k in zip((a, b, c, d), ("tt", "ti", "it", "ii")):
            _close(y, z[k], 5e-2)


def test_full_dims_factify_shapes_vs_oracle():
    """BASELINE shapes (text 128 x 768, image 197 x 768) at B=2, fp32, vs the CPU oracle."""
    g = torch.Generator().manual_seed(3)
    X = [torch.randn(2, 128, 768, generator=g), torch.randn(2, 197, 768, generator=g),
         torch.randn(2, 128, 768, generator=g), torch.randn(2, 197, 768, generator=g)]
    m = MisinformationDetectionModel(text_input_dim=768, image_input_dim=768).to(DEV).eval()
    P = {n: p.detach().cpu() for n, p in m.named_parameters()}
    with torch.no_grad():
        (a, b), (c, d) = m(*(x.to(DEV) for x in X))
        (ar, br), (cr, dr) = OF.model_forward(P, *X, num_heads=8)
    for y, r in zip((a, b, c, d), (ar, br, cr, dr)):
        _close(y, r, 1e-4)


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_two_stream_head_matches_serial(monkeypatch, precision):
    """The head's claim-text / claim-image halves on two HIP streams (fusion._fwd_two_streams /
    _bwd_two_streams) against MMFD_SERIAL_HEAD=1 at full head dims (E=256, 8 heads, text 128 and
    image 197 rows, B=8), train mode with dropout 0.1: fp32 logits and every gradient bit-identical
    (the evidence dk|dv sum is the same fp32 addition the serial in-kernel accumulation does); bf16:
    the two-stream sum rounds the second path's dk|dv to bf16 once more, so the logits and the input
    gradients agree to 5e-2 in relative norm (small parameter gradients are bf16 noise there)."""
    g = torch.Generator().manual_seed(11)
    X = [torch.randn(8, 128, 768, generator=g), torch.randn(8, 197, 768, generator=g),
         torch.randn(8, 128, 768, generator=g), torch.randn(8, 197, 768, generator=g)]
    m = MisinformationDetectionModel(text_input_dim=768, image_input_dim=768, dropout=0.1).to(DEV).train()
    if precision == "bf16":
        m.set_precision("bf16")
    R = [torch.randn(8, 3, generator=g).to(DEV) for _ in range(4)]

    def run(serial):
        monkeypatch.setenv("MMFD_SERIAL_HEAD", "1" if serial else "0")
        m.manual_seed(77)
        m.zero_grad(set_to_none=True)
        Xg = [x.to(DEV).requires_grad_(True) for x in X]
        (a, b), (c, d) = m(*Xg)
        sum((y * r).sum() for y, r in zip((a, b, c, d), R)).backward()
        torch.cuda.synchronize()
        return ([y.detach().clone() for y in (a, b, c, d)], [x.grad.clone() for x in Xg],
                {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None})

    ys, xs, ps = run(True)
    yt, xt, pt = run(False)
    assert ps.keys() == pt.keys()
    if precision == "fp32":
        for s, t in list(zip(ys, yt)) + list(zip(xs, xt)) + [(ps[n], pt[n]) for n in ps]:
            assert torch.equal(s, t)
    else:
        for s, t in list(zip(ys, yt)) + list(zip(xs, xt)):
            assert (s.float() - t.float()).norm().item() <= 5e-2 * s.float().norm().item()
