"""TEST INFRASTRUCTURE ONLY (oracle). Imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg — never by the product path.

CPU restatement (plain torch functional ops, fp32/fp64) of the reference fusion classifier:
  src/model/layers.py:5-58      MLP, MultiHeadAttention (eager branch; SDPA branch is the same math)
  src/model/model.py:6-121      MultiViewClaimRepresentation (multimodal + unimodal branches)
  src/model/model.py:124-237    CrossAttentionEvidenceConditioning (4 paths)
  src/model/model.py:240-347    ClassificationModule (4-path / factify)
  src/model/model.py:350-468    MisinformationDetectionModel (text_only / factify / 4-path dispatch)
Parameters are a dict keyed by the reference's state_dict names. Dropout is applied through a
`drop(site, x)` callback so that train-mode parity can use the exact counter-based masks of the HIP
kernels (oracle/dropout_hash.py); with drop=None the oracle is the eval-mode reference.
Pinned against fixtures produced by the reference itself (tests/golden/make_golden.py).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def _lin(P, name, x):
    return F.linear(x, P[name + ".weight"], P[name + ".bias"])


def _ln(P, name, x, eps=1e-5):
    return F.layer_norm(x, (x.shape[-1],), P[name + ".weight"], P[name + ".bias"], eps)


def _drop(drop, site, x):
    return x if drop is None else drop(site, x)


def mha(Q, K, V, P, out_name, H, drop=None, site=""):
    """layers.py:36-58: per-head softmax(QK^T/sqrt(hd)) V, attention dropout, out_proj."""
    B, T, D = Q.shape
    hd = D // H
    q = Q.reshape(B, T, H, hd).transpose(1, 2)
    k = K.reshape(B, -1, H, hd).transpose(1, 2)
    v = V.reshape(B, -1, H, hd).transpose(1, 2)
    s = torch.matmul(q, k.transpose(-1, -2)) / (hd ** 0.5)
    a = torch.softmax(s, dim=-1)
    a = _drop(drop, site + ".attn", a)
    ctx = torch.matmul(a, v).transpose(1, 2).reshape(B, T, D)
    return _lin(P, out_name, ctx)


def mlp(P, name, x, drop=None, site=""):
    """layers.py:12-18: Linear -> GELU(erf) -> Dropout -> Linear -> Dropout."""
    h = F.gelu(_lin(P, name + ".net.0", x))
    h = _drop(drop, site + ".h", h)
    y = _lin(P, name + ".net.3", h)
    return _drop(drop, site + ".out", y)


def representation(P, X_t, X_i, H, drop=None, pre="representation"):
    """model.py:56-121."""
    r = pre + "."
    Xt = _lin(P, r + "text_proj", X_t) if X_t is not None else None
    Xi = _lin(P, r + "image_proj", X_i) if X_i is not None else None
    if Xt is not None:
        tQ, tK, tV = (_lin(P, r + n, Xt) for n in ("text_WQ", "text_WK", "text_WV"))
    if Xi is not None:
        iQ, iK, iV = (_lin(P, r + n, Xi) for n in ("image_WQ", "image_WK", "image_WV"))
    if Xt is not None and Xi is None:  # :83-90
        Ht = _ln(P, r + "text_self_ln1", Xt + mha(tQ, tK, tV, P, r + "text_self_attn_out", H, drop, r + "text.self"))
        Ht = _ln(P, r + "text_self_ln2", Ht + mlp(P, r + "text_mlp", Ht, drop, r + "text.mlp"))
        return Ht, None
    if Xi is not None and Xt is None:  # :93-100
        Hi = _ln(P, r + "image_self_ln1", Xi + mha(iQ, iK, iV, P, r + "image_self_attn_out", H, drop, r + "image.self"))
        Hi = _ln(P, r + "image_self_ln2", Hi + mlp(P, r + "image_mlp", Hi, drop, r + "image.mlp"))
        return None, Hi
    # :103-121
    Ht = _ln(P, r + "text_self_ln1", Xt + mha(tQ, tK, tV, P, r + "text_self_attn_out", H, drop, r + "text.self"))
    Ct = _ln(P, r + "text_cross_ln1", Ht + mha(Ht, tK, tV, P, r + "text_cross_attn_out", H, drop, r + "text.cross"))
    Ct = _ln(P, r + "text_cross_ln2", Ct + mlp(P, r + "text_mlp", Ct, drop, r + "text.mlp"))
    Hi = _ln(P, r + "image_self_ln1", Xi + mha(iQ, iK, iV, P, r + "image_self_attn_out", H, drop, r + "image.self"))
    Ci = _ln(P, r + "image_cross_ln1", Hi + mha(Hi, iK, iV, P, r + "image_cross_attn_out", H, drop, r + "image.cross"))
    Ci = _ln(P, r + "image_cross_ln2", Ci + mlp(P, r + "image_mlp", Ci, drop, r + "image.mlp"))
    return Ct, Ci


def _path(P, c, Hq, wq, E, key, val, out, ln1, ln2, mlp_name, H, drop, site):
    a = mha(_lin(P, c + wq, Hq), _lin(P, c + key, E), _lin(P, c + val, E), P, c + out, H, drop, site)
    a = _ln(P, c + ln1, Hq + a)
    return _ln(P, c + ln2, a + mlp(P, c + mlp_name, a, drop, site + ".mlp"))


def cross_attn(P, Ht, Hi, Et, Ei, H, drop=None, pre="cross_attn"):
    """model.py:172-237 (the Q projection and evidence K/V are recomputed per path in the
    reference; they are deterministic, so computing them per path here is the same value)."""
    c = pre + "."
    Stt = Sti = Sit = Sii = None
    if Ht is not None and Et is not None:
        Stt = _path(P, c, Ht, "text_WQ", Et, "text_evidence_key", "text_evidence_value", "text_text_out",
                    "text_text_ln1", "text_text_ln2", "text_mlp", H, drop, c + "tt")
    if Ht is not None and Ei is not None:
        Sti = _path(P, c, Ht, "text_WQ", Ei, "image_evidence_key", "image_evidence_value", "text_image_out",
                    "text_image_ln1", "text_image_ln2", "text_mlp", H, drop, c + "ti")
    if Hi is not None and Et is not None:
        Sit = _path(P, c, Hi, "image_WQ", Et, "text_evidence_key", "text_evidence_value", "image_text_out",
                    "image_text_ln1", "image_text_ln2", "image_mlp", H, drop, c + "it")
    if Hi is not None and Ei is not None:
        Sii = _path(P, c, Hi, "image_WQ", Ei, "image_evidence_key", "image_evidence_value", "image_image_out",
                    "image_image_ln1", "image_image_ln2", "image_mlp", H, drop, c + "ii")
    return (Stt, Sti), (Sit, Sii)


def _head(P, name, x, n_hidden, drop, site):
    """nn.Sequential(Linear, ReLU, Dropout, Linear[, ReLU, Dropout, Linear])"""
    idx = 0
    for layer in range(n_hidden):
        x = torch.relu(_lin(P, f"{name}.{idx}", x))
        x = _drop(drop, f"{site}.d{layer}", x)
        idx += 3
    return _lin(P, f"{name}.{idx}", x)


def classifier(P, S_t, S_i, factify, drop=None, pre="classifier"):
    """model.py:290-347."""
    c = pre + "."
    if factify:
        feats = [s.mean(dim=1) for s in (*S_t, *S_i) if s is not None]
        return _head(P, c + "unified_mlp", torch.cat(feats, dim=1), 2, drop, c + "unified"), None
    names = [("mlp_text_given_text", S_t[0]), ("mlp_text_given_image", S_t[1]),
             ("mlp_image_given_text", S_i[0]), ("mlp_image_given_image", S_i[1])]
    ys = [None if s is None else _head(P, c + n, s.mean(dim=1), 1, drop, c + n) for n, s in names]
    return (ys[0], ys[1]), (ys[2], ys[3])


def model_forward(P, X_t=None, X_i=None, E_t=None, E_i=None, *, num_heads=8, factify=False, text_only=False,
                  drop=None):
    """model.py:426-468."""
    if text_only:
        Ht, _ = representation(P, X_t, None, num_heads, drop)
        (Stt, _), _ = cross_attn(P, Ht, None, E_t, None, num_heads, drop)
        return _head(P, "text_classifier", Stt.mean(dim=1), 2, drop, "text_classifier"), None
    Ht, Hi = representation(P, X_t, X_i, num_heads, drop)
    S_t, S_i = cross_attn(P, Ht, Hi, E_t, E_i, num_heads, drop)
    if factify:
        return classifier(P, S_t, S_i, True, drop)
    return classifier(P, S_t, S_i, False, drop)


def path_loss(outputs, labels):
    """train.py:161-169: sum over available paths of CrossEntropyLoss(y_i, labels[:, i])."""
    (ytt, yti), (yit, yii) = outputs
    total, per = 0.0, []
    for i, y in enumerate((ytt, yti, yit, yii)):
        if y is None:
            per.append(None)
            continue
        li = F.cross_entropy(y, labels[:, i])
        per.append(li)
        total = total + li
    return total, per


def init_params_like_reference(names_shapes, seed):
    """A deterministic, reference-independent weight recipe (used for full-size fixtures whose
    weights are too large to commit): W ~ N(0, 0.02) per tensor from a per-name generator,
    LayerNorm weights 1 + N(0, 0.02)."""
    import zlib

    P = {}
    for name, shape in names_shapes:
        g = torch.Generator().manual_seed(seed * 1000003 + zlib.crc32(name.encode()))
        t = torch.randn(*shape, generator=g) * 0.02
        if ("ln" in name.split(".")[-2] or "LayerNorm" in name or "layernorm" in name) and name.endswith("weight"):
            t = t + 1.0
        P[name] = t
    return P


def xavier_like_reference(names_shapes, seed):
    """Mirror of _initialize_weights (model.py:416-424) draw-order-free: xavier_uniform per Linear
    weight with a per-name generator, zero bias, LN 1/0."""
    import zlib

    P = {}
    for name, shape in names_shapes:
        if len(shape) == 2:
            g = torch.Generator().manual_seed(seed * 1000003 + zlib.crc32(name.encode()))
            a = math.sqrt(6.0 / (shape[0] + shape[1]))
            P[name] = (torch.rand(*shape, generator=g) * 2 - 1) * a
        elif name.endswith("weight"):
            P[name] = torch.ones(*shape)
        else:
            P[name] = torch.zeros(*shape)
    return P
