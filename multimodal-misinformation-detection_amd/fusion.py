"""The fusion classifier (reference src/model/model.py + layers.py) as an explicit forward and a
hand-written backward over HIP kernels.

Forward follows model.py:426-468 exactly, including its quirks:
  * the representation's "cross" attention uses the unprojected H as Q against the same
    modality's K/V (model.py:106, 115);
  * no padding mask anywhere in the head (layers.py:51); mean pooling over all positions;
  * text_self_ln2 / image_self_ln2 are only used by the unimodal branches (model.py:89, 99).
MI355X-specific restructuring (same values): Q/K/V of a modality are one fused GEMM (N = 3E); the
evidence K and V are one GEMM (N = 2E) computed once per modality instead of once per path, and
the per-path Q projections once per claim modality (model.py:188/201, 189-190/215-216, 202-203/
228-229, 214/227 recompute identical values); every attention output projection carries the
residual add in its GEMM epilogue; dropout masks are generated in the epilogues.
"""
from __future__ import annotations

import os

import torch

from . import blocks as Bk
from . import kernels as K


class HeadConfig:
    def __init__(self, embed_dim, num_heads, factify=False, text_only=False, ln_eps=1e-5):
        self.E = embed_dim
        self.H = num_heads
        self.factify = factify
        self.text_only = text_only
        self.eps = ln_eps


# -------------------------------------------------------------------------------------------------
# attention block: y = LN(res + out_proj(MHA(q, k, v)))
# -------------------------------------------------------------------------------------------------
# Split-operand fp32 mode (Bk.StepCtx.planes): every GEMM input of the head is split into its bf16
# planes once, by its producer where one can (attention output, GEMM epilogue, LayerNorm forward /
# backward), else by one split3 pass, and the planes are kept for the weight-gradient GEMM; every
# output gradient is split once for its data- and weight-gradient GEMMs. All planes are None in
# bf16 / fp32-MFMA mode.
def _attn_ln_fwd(ctx, cfg, q, k, v, res2d, out_name, ln_name, site, want_planes=False):
    """(y, y planes or None, state)"""
    B, Lq, _ = q.shape
    op = Bk.new_planes(ctx, B * Lq, q.shape[2], q.device)
    o, lse = K.attn_fwd(q, k, v, cfg.H, o_planes=op, **ctx.attn_drop(site + ".attn", q, k, cfg.H))
    s, _ = Bk.linear(ctx, Bk.as2d(o), out_name, residual=res2d, xp=op)
    y, mean, rstd, yp = Bk.layernorm_planes(ctx, s, ln_name, cfg.eps, want=want_planes)
    return y, yp, (q, k, v, o, op, lse, s, mean, rstd, out_name, ln_name, site)


def _attn_ln_out_bwd(ctx, dy2d, st):
    """LayerNorm + output-projection backward of an attention block: (ds, do)"""
    q, k, v, o, op, lse, s, mean, rstd, out_name, ln_name, site = st
    if op is not None:
        ds, _, dsp = Bk.layernorm_bwd_planes(ctx, dy2d, s, ln_name, mean, rstd)
    else:
        (ds, _), dsp = Bk.layernorm_bwd(ctx, dy2d, s, ln_name, mean, rstd), None
    ctx.lin_grads([out_name], ds, Bk.as2d(o), dsp, op)
    do = Bk.linear_dx(ctx, ds, out_name, dyp=dsp).view(o.shape)
    return ds, do


def _attn_ln_bwd(ctx, cfg, dy2d, st, *, dq=None, acc_dq=False, dk=None, dv=None, acc_dkv=False, dqkv_planes=None):
    """Returns ds (the gradient of the residual input); writes/accumulates dq, dk, dv."""
    q, k, v, o, op, lse, s, mean, rstd, out_name, ln_name, site = st
    ds, do = _attn_ln_out_bwd(ctx, dy2d, st)
    K.attn_bwd(q, k, v, o, lse, do, cfg.H, dq=dq, dk=dk, dv=dv, accumulate_dq=acc_dq, accumulate_dkv=acc_dkv,
               dqkv_planes=dqkv_planes, **ctx.attn_drop(site + ".attn"))
    return ds


# -------------------------------------------------------------------------------------------------
# representation (model.py:56-121)
# -------------------------------------------------------------------------------------------------
def _repr_modality_fwd(ctx, cfg, Xin, m, unimodal):
    r = "representation."
    B, L, _ = Xin.shape
    E = cfg.E
    x2d = Bk.as2d(Xin)
    xinp = ctx.planes(x2d)
    # X feeds the QKV GEMM (planes from the projection's epilogue) and the self-attention residual
    Xp = Bk.out_planes(ctx, B * L, E, (), Xin.device)[0] if xinp is not None else None
    X, _ = Bk.linear(ctx, x2d, r + f"{m}_proj", xp=xinp, out_planes=Xp)
    qkv = Bk.linear_packed(ctx, X, [r + f"{m}_WQ", r + f"{m}_WK", r + f"{m}_WV"], xp=Xp).view(B, L, 3 * E)
    q, k, v = qkv[..., :E], qkv[..., E:2 * E], qkv[..., 2 * E:]
    sp = xinp is not None
    Hh, Hp, st1 = _attn_ln_fwd(ctx, cfg, q, k, v, X, r + f"{m}_self_attn_out", r + f"{m}_self_ln1", r + f"{m}.self",
                               want_planes=unimodal and sp)
    st = dict(Xin=Xin, xinp=xinp, X=X, Xp=Xp, qkv=qkv, st1=st1, st2=None, m=m)
    if unimodal:  # model.py:83-100: self-attention, then MLP + self_ln2
        Y, Yp, st["st3"] = Bk.mlp_ln_fwd(ctx, Hh, r + f"{m}_mlp", r + f"{m}_self_ln2", r + f"{m}.mlp", cfg.eps, ap=Hp,
                                         want_planes=sp)
        return Y.view(B, L, E), Yp, st
    Hv = Hh.view(B, L, E)
    C, Cp, st["st2"] = _attn_ln_fwd(ctx, cfg, Hv, k, v, Hh, r + f"{m}_cross_attn_out", r + f"{m}_cross_ln1",
                                    r + f"{m}.cross", want_planes=sp)
    Y, Yp, st["st3"] = Bk.mlp_ln_fwd(ctx, C, r + f"{m}_mlp", r + f"{m}_cross_ln2", r + f"{m}.mlp", cfg.eps, ap=Cp,
                                     want_planes=sp)
    return Y.view(B, L, E), Yp, st


def _repr_modality_bwd(ctx, cfg, dY2d, st, need_dxin, out=None):
    r = "representation."
    m = st["m"]
    E = cfg.E
    qkv = st["qkv"]
    B, L, _ = qkv.shape
    dqkv = torch.empty_like(qkv)
    # the packed dQ|dK|dV's planes come from the last attention backward that writes it
    dqkvp = Bk.new_planes(ctx, B * L, 3 * E, qkv.device) if st["Xp"] is not None else None
    dC = Bk.mlp_ln_bwd(ctx, dY2d, st["st3"])
    if st["st2"] is not None:
        q2, k2, v2, o2, _, lse2, _, _, _, _, _, site2 = st["st2"]
        ds2, do2 = _attn_ln_out_bwd(ctx, dC, st["st2"])      # ds2: dH (residual part)
        # dq of the cross attention goes straight into dH (= ds2), dk/dv start dQKV's K|V blocks
        K.attn_bwd(q2, k2, v2, o2, lse2, do2, cfg.H, dq=ds2.view(B, L, E), dk=dqkv[..., E:2 * E],
                   dv=dqkv[..., 2 * E:], accumulate_dq=True, accumulate_dkv=False, **ctx.attn_drop(site2 + ".attn"))
        dX = _attn_ln_bwd(ctx, cfg, ds2, st["st1"], dq=dqkv[..., :E], dk=dqkv[..., E:2 * E], dv=dqkv[..., 2 * E:],
                          acc_dkv=True, dqkv_planes=dqkvp)
    else:
        dX = _attn_ln_bwd(ctx, cfg, dC, st["st1"], dq=dqkv[..., :E], dk=dqkv[..., E:2 * E], dv=dqkv[..., 2 * E:],
                          dqkv_planes=dqkvp)
    dqkv2 = Bk.as2d(dqkv)
    names = [r + f"{m}_WQ", r + f"{m}_WK", r + f"{m}_WV"]
    ctx.lin_grads(names, dqkv2, st["X"], dqkvp, st["Xp"])
    Wp, _ = ctx.w_packed(names)
    Bk.linear_dx(ctx, dqkv2, Wp, out=dX, beta=1.0, dyp=dqkvp)  # dX += dQKV [WQ;WK;WV]
    dXp = ctx.planes(dX) if st["xinp"] is not None else None
    ctx.lin_grads([r + f"{m}_proj"], dX, Bk.as2d(st["Xin"]), dXp, st["xinp"])
    if not need_dxin:
        return None
    return Bk.linear_dx(ctx, dX, r + f"{m}_proj", out=out, dyp=dXp).view(st["Xin"].shape)


# -------------------------------------------------------------------------------------------------
# evidence conditioning (model.py:172-237)
# -------------------------------------------------------------------------------------------------
PATHS = [  # (claim modality, evidence modality, path tag, out proj, ln prefix)
    ("text", "text", "tt", "text_text"),
    ("text", "image", "ti", "text_image"),
    ("image", "text", "it", "image_text"),
    ("image", "image", "ii", "image_image"),
]
PATH_OF = {(p[0], p[1]): p for p in PATHS}
OTHER = {"text": "image", "image": "text"}

_HEAD_SIDE = {}


def _two_streams(*xs):
    """whether the head's claim-text and claim-image halves run on two HIP streams: both
    modalities present (the full four-path head) on a GPU, unless MMFD_SERIAL_HEAD=1"""
    return (all(x is not None for x in xs) and xs[0].is_cuda and os.environ.get("MMFD_SERIAL_HEAD") != "1")


def _head_stream(device):
    s = _HEAD_SIDE.get(device.index)
    if s is None:
        s = _HEAD_SIDE[device.index] = torch.cuda.Stream(device=device)
    return s


def _publish(stream, *ts):
    """mark tensors one head stream hands to the other as used by `stream` (record_stream), so the
    caching allocator does not give their blocks to a later allocation of the producing stream
    before the reader's queued kernels have run. (The side stream also always starts with
    side.wait_stream(main), ADVICE r3: this keeps the hand-off safe without relying on that.)"""
    for t in ts:
        if torch.is_tensor(t):
            t.record_stream(stream)


def _event():
    e = torch.cuda.Event()
    e.record()
    return e


def _kv_fwd(ctx, cfg, Em, m, EP):
    """evidence K|V of modality m: one GEMM (N = 2E) shared by both paths that read it; the
    evidence's planes go to EP[m] for the weight-gradient GEMM"""
    c = "cross_attn."
    B, L, _ = Em.shape
    e2d = Bk.as2d(Em)
    EP[m] = ctx.planes(e2d)
    return Bk.linear_packed(ctx, e2d, [c + f"{m}_evidence_key", c + f"{m}_evidence_value"], xp=EP[m]
                            ).view(B, L, 2 * cfg.E)


def _q_fwd(ctx, cfg, H, Hp, m):
    """the claim modality's conditioning Q projection, shared by its two paths"""
    B, L, _ = H.shape
    return Bk.linear(ctx, Bk.as2d(H), f"cross_attn.{m}_WQ", xp=Hp)[0].view(B, L, cfg.E)


def _path_fwd(ctx, cfg, path, q, kv, H):
    """one conditioning path (model.py:186-195 and its three siblings): LN(H + out(MHA(Q, K, V))),
    then the claim modality's MLP block with the path's ln2"""
    hm, em, tag, name = path
    c = "cross_attn."
    E = cfg.E
    a, ap, s1 = _attn_ln_fwd(ctx, cfg, q, kv[..., :E], kv[..., E:], Bk.as2d(H), c + f"{name}_out",
                             c + f"{name}_ln1", c + tag, want_planes=True)
    S, _, s2 = Bk.mlp_ln_fwd(ctx, a, c + f"{hm}_mlp", c + f"{name}_ln2", c + tag + ".mlp", cfg.eps, ap=ap)
    return S.view(H.shape), (s1, s2)


def _cond_fwd(ctx, cfg, Hs, HP, Es):
    Q, KV, EP, out, st = {}, {}, {}, {}, {}
    for m in ("text", "image"):
        if Hs.get(m) is not None and any(Es.get(e) is not None for e in ("text", "image")):
            Q[m] = _q_fwd(ctx, cfg, Hs[m], HP.get(m), m)
        if Es.get(m) is not None and any(Hs.get(x) is not None for x in ("text", "image")):
            KV[m] = _kv_fwd(ctx, cfg, Es[m], m, EP)
    for path in PATHS:
        hm, em, tag, _ = path
        if Hs.get(hm) is None or Es.get(em) is None:
            continue
        out[tag], st[tag] = _path_fwd(ctx, cfg, path, Q[hm], KV[em], Hs[hm])
    return out, dict(Q=Q, KV=KV, st=st, Hs=Hs, HP=HP, Es=Es, EP=EP)


def _path_bwd(ctx, cfg, path, dS, cst, dH, dQ, dKV):
    """backward of one conditioning path: the residual gradient is summed into dH[claim modality],
    the attention's dq into dQ[claim modality] and its dk|dv into dKV[evidence modality] (each
    written by the first path that reaches it, accumulated by the second)"""
    hm, em, tag, _ = path
    E = cfg.E
    s1, s2 = cst["st"][tag]
    da = Bk.mlp_ln_bwd(ctx, Bk.as2d(dS[tag]), s2)
    q, k, v, o, _, lse, _, _, _, _, _, site = s1
    ds, do = _attn_ln_out_bwd(ctx, da, s1)
    # residual gradient into H, summed over the claim modality's two paths
    if hm in dH:
        K.axpby(1.0, dH[hm], 1.0, ds, out=dH[hm])
    else:
        dH[hm] = ds
    first_q = hm not in dQ
    first_kv = em not in dKV
    if first_q:
        dQ[hm] = torch.empty_like(q)
    if first_kv:
        dKV[em] = torch.empty_like(cst["KV"][em])
    K.attn_bwd(q, k, v, o, lse, do, cfg.H, dq=dQ[hm], dk=dKV[em][..., :E], dv=dKV[em][..., E:],
               accumulate_dq=not first_q, accumulate_dkv=not first_kv, **ctx.attn_drop(site + ".attn"))


def _q_bwd(ctx, cfg, hm, dq, cst, dH):
    """WQ gradients and dH[hm] += dQ WQ"""
    dq2 = Bk.as2d(dq)
    name = f"cross_attn.{hm}_WQ"
    hp = cst["HP"].get(hm)
    dqp = ctx.planes(dq2) if hp is not None else None
    ctx.lin_grads([name], dq2, Bk.as2d(cst["Hs"][hm]), dqp, hp)
    Bk.linear_dx(ctx, dq2, name, out=dH[hm], beta=1.0, dyp=dqp)


def _kv_bwd(ctx, cfg, em, dkv, cst, need, out=None):
    """evidence K|V weight gradients; returns dE (or None when not needed)"""
    names = [f"cross_attn.{em}_evidence_key", f"cross_attn.{em}_evidence_value"]
    dkv2 = Bk.as2d(dkv)
    ep = cst["EP"].get(em)
    dkvp = ctx.planes(dkv2) if ep is not None else None
    ctx.lin_grads(names, dkv2, Bk.as2d(cst["Es"][em]), dkvp, ep)
    if not need:
        return None
    Wp, _ = ctx.w_packed(names)
    return Bk.linear_dx(ctx, dkv2, Wp, out=out, dyp=dkvp).view(cst["Es"][em].shape)


def _cond_bwd(ctx, cfg, dS, cst, need_dE, out_dE=None):
    """dS: tag -> [B, L, E] grads. Returns (dH per claim modality (2-D), dE per evidence modality)."""
    dH, dQ, dKV = {}, {}, {}
    for path in PATHS:
        if path[2] in cst["st"]:
            _path_bwd(ctx, cfg, path, dS, cst, dH, dQ, dKV)
    for hm, dq in dQ.items():
        _q_bwd(ctx, cfg, hm, dq, cst, dH)
    dE = {}
    for em, dkv in dKV.items():
        d = _kv_bwd(ctx, cfg, em, dkv, cst, need_dE.get(em), (out_dE or {}).get(em))
        if d is not None:
            dE[em] = d
    return dH, dE


def _fwd_two_streams(ctx, cfg, Xs, Es):
    """Representation + conditioning with the claim-text half (representation, Q, paths tt and ti)
    on the current stream and the claim-image half (it, ii) on a second one. The head's GEMMs have
    N = E = 256 and K = 256-1024: one 256x256 tile column over B*L rows leaves half the CUs idle
    (128 tiles for text, 197 for image), and the two halves only meet at the evidence K|V, which
    each stream computes first and publishes by an event. Same kernels and values as _cond_fwd."""
    main = torch.cuda.current_stream()
    side = _head_stream(Xs["text"].device)
    side.wait_stream(main)
    streams = {"text": main, "image": side}
    Hs, HP, EP, rst, Q, KV, ev, out, st = {}, {}, {}, {}, {}, {}, {}, {}, {}
    for m in ("text", "image"):
        with torch.cuda.stream(streams[m]):
            KV[m] = _kv_fwd(ctx, cfg, Es[m], m, EP)
            ev[m] = _event()
    for m in ("text", "image"):
        with torch.cuda.stream(streams[m]):
            Hs[m], HP[m], rst[m] = _repr_modality_fwd(ctx, cfg, Xs[m], m, unimodal=False)
            Q[m] = _q_fwd(ctx, cfg, Hs[m], HP[m], m)
            for em in (m, OTHER[m]):  # own evidence first: the other stream's K|V may still be running
                if em != m:
                    torch.cuda.current_stream().wait_event(ev[em])
                path = PATH_OF[(m, em)]
                out[path[2]], st[path[2]] = _path_fwd(ctx, cfg, path, Q[m], KV[em], Hs[m])
    main.wait_stream(side)
    _publish(side, KV["text"])
    _publish(main, KV["image"], out["it"], out["ii"], Hs["image"])
    return Hs, rst, {t: out[t] for t in ("tt", "ti", "it", "ii")}, dict(Q=Q, KV=KV, st=st, Hs=Hs, HP=HP, Es=Es,
                                                                         EP=EP)


def _bwd_two_streams(ctx, cfg, dS, state, need_dX, need_e, outs):
    """head_backward's conditioning + representation part on the streams of _fwd_two_streams. Each
    stream accumulates its own paths' dk|dv per evidence modality; after both have published theirs
    (events), the evidence modality's stream sums the two (fp32: the same value as the serial
    in-kernel accumulation) and runs the evidence K|V gradients."""
    cst = state["cst"]
    main = torch.cuda.current_stream()
    side = _head_stream(dS["tt"].device)
    side.wait_stream(main)
    _publish(side, dS["it"], dS["ii"])
    streams = {"text": main, "image": side}
    dKVs, ev, dX, dE = {}, {}, {}, {}
    for m in ("text", "image"):
        with torch.cuda.stream(streams[m]):
            dH, dQ, dKV = {}, {}, {}
            for path in PATHS:
                if path[0] == m:
                    _path_bwd(ctx, cfg, path, dS, cst, dH, dQ, dKV)
            dKVs[m] = dKV
            ev[m] = _event()
            _q_bwd(ctx, cfg, m, dQ[m], cst, dH)
            dX[m] = _repr_modality_bwd(ctx, cfg, dH[m], state["rst"][m], need_dX[m], out=outs[m])
    for em in ("text", "image"):
        with torch.cuda.stream(streams[em]):
            torch.cuda.current_stream().wait_event(ev[OTHER[em]])
            # claim-text path first, as the serial PATHS order accumulates
            dkv = dKVs[em][em]
            K.axpby(1.0, dKVs["text"][em], 1.0, dKVs["image"][em], out=dkv)
            dE[em] = _kv_bwd(ctx, cfg, em, dkv, cst, need_e[em], outs["E" + em])
    main.wait_stream(side)
    _publish(side, dKVs["text"].get("image"))
    _publish(main, dKVs["image"].get("text"), dX.get("image"), dE.get("image"))
    return dX, dE


# -------------------------------------------------------------------------------------------------
# classifiers (model.py:240-347, 393-403)
# -------------------------------------------------------------------------------------------------
def _mlp_head_fwd(ctx, x2d, name, n_hidden, site):
    acts = [x2d]
    pres = []
    idx = 0
    h = x2d
    for layer in range(n_hidden):
        h, pre = Bk.linear(ctx, h, f"{name}.{idx}", act=K.ACT_RELU, keep_aux=True, drop_site=f"{site}.d{layer}")
        acts.append(h)
        pres.append(pre)
        idx += 3
    y, _ = Bk.linear(ctx, h, f"{name}.{idx}", out_dtype=torch.float32)
    return y, (acts, pres, name, n_hidden, site)


def _mlp_head_bwd(ctx, dy, st):
    acts, pres, name, n_hidden, site = st
    g = dy if ctx.dt == torch.float32 else K.cast(dy, ctx.dt)
    idx = 3 * n_hidden
    ctx.lin_grads([f"{name}.{idx}"], g, acts[-1])
    for layer in reversed(range(n_hidden)):
        # d(pre) = dX(next) * relu'(pre) * dropout mask
        g = Bk.linear_dx(ctx, g, f"{name}.{idx}", act=K.ACT_RELU_BWD, aux=pres[layer], drop_site=f"{site}.d{layer}")
        idx -= 3
        ctx.lin_grads([f"{name}.{idx}"], g, acts[layer])
    return Bk.linear_dx(ctx, g, f"{name}.{idx}")


CLS_NAMES = {"tt": "mlp_text_given_text", "ti": "mlp_text_given_image", "it": "mlp_image_given_text",
             "ii": "mlp_image_given_image"}


# -------------------------------------------------------------------------------------------------
# whole head
# -------------------------------------------------------------------------------------------------
def head_forward(ctx, cfg: HeadConfig, X_t, X_i, E_t, E_i):
    """Returns (outputs, state). outputs: dict tag -> fp32 logits ('pred' for factify/text_only)."""
    dt = ctx.dt
    cast_in = lambda x: None if x is None else (x if x.dtype == dt else K.cast(x, dt))  # noqa: E731
    X_t, X_i, E_t, E_i = (cast_in(x) for x in (X_t, X_i, E_t, E_i))
    if cfg.text_only:
        X_i = E_i = None
    Hs, rst = {}, {}
    uni = (X_t is None) != (X_i is None) or cfg.text_only
    Es = {"text": E_t, "image": E_i}
    two = not uni and _two_streams(X_t, X_i, E_t, E_i)
    if two:
        Hs, rst, S, cst = _fwd_two_streams(ctx, cfg, {"text": X_t, "image": X_i}, Es)
    else:
        HP = {}
        for m, x in (("text", X_t), ("image", X_i)):
            if x is not None:
                Hs[m], HP[m], rst[m] = _repr_modality_fwd(ctx, cfg, x, m, unimodal=uni)
        S, cst = _cond_fwd(ctx, cfg, Hs, HP, Es)
    pooled, hst, outs = {}, {}, {}
    if cfg.text_only:
        p = K.seq_mean_fwd(S["tt"])
        outs["pred"], hst["pred"] = _mlp_head_fwd(ctx, p, "text_classifier", 2, "text_classifier")
        pooled["tt"] = p
    elif cfg.factify:
        tags = [t for t in ("tt", "ti", "it", "ii") if t in S]
        B = S[tags[0]].shape[0]
        cat = torch.empty((B, cfg.E * len(tags)), device=S[tags[0]].device, dtype=dt)
        for j, t in enumerate(tags):
            K.seq_mean_fwd(S[t], out=cat[:, j * cfg.E:(j + 1) * cfg.E])
        outs["pred"], hst["pred"] = _mlp_head_fwd(ctx, cat, "classifier.unified_mlp", 2, "classifier.unified")
        hst["tags"] = tags
    else:
        for t in ("tt", "ti", "it", "ii"):
            if t in S:
                p = K.seq_mean_fwd(S[t])
                name = "classifier." + CLS_NAMES[t]
                outs[t], hst[t] = _mlp_head_fwd(ctx, p, name, 1, name)
    state = dict(rst=rst, cst=cst, S=S, hst=hst, two=two, shapes={m: x.shape for m, x in (("text", X_t), ("image", X_i))
                                                          if x is not None})
    return outs, state


def head_backward(ctx, cfg: HeadConfig, douts, state, need_dX=(True, True), need_dE=(True, True), outs=None):
    """douts: dict tag -> fp32 grad of logits. Returns dX_t, dX_i, dE_t, dE_i (compute dtype or None).
    `outs` (optional 4-tuple of 2-D compute-dtype buffers or None) receive them in place: the halves
    of the stacked claim/evidence encoder-output gradient (FusionTrainer, no split/concat copies)."""
    outs = outs or (None, None, None, None)
    S = state["S"]
    hst = state["hst"]
    dS = {}
    if cfg.text_only or cfg.factify:
        dcat = _mlp_head_bwd(ctx, douts["pred"], hst["pred"])
        if cfg.text_only:
            dS["tt"] = K.seq_mean_bwd(dcat, S["tt"].shape[1])
        else:
            for j, t in enumerate(hst["tags"]):
                dS[t] = K.seq_mean_bwd(dcat[:, j * cfg.E:(j + 1) * cfg.E], S[t].shape[1])
    else:
        for t, st in hst.items():
            dp = _mlp_head_bwd(ctx, douts[t], st)
            dS[t] = K.seq_mean_bwd(dp, S[t].shape[1])
    need_e = {"text": need_dE[0], "image": need_dE[1]}
    if state.get("two"):
        dX, dE = _bwd_two_streams(ctx, cfg, dS, state, {"text": need_dX[0], "image": need_dX[1]}, need_e,
                                  {"text": outs[0], "image": outs[1], "Etext": outs[2], "Eimage": outs[3]})
        return dX.get("text"), dX.get("image"), dE.get("text"), dE.get("image")
    dH, dE = _cond_bwd(ctx, cfg, dS, state["cst"], need_e, out_dE={"text": outs[2], "image": outs[3]})
    dX = {}
    for m, st in state["rst"].items():
        need = need_dX[0] if m == "text" else need_dX[1]
        if m in dH:
            dX[m] = _repr_modality_bwd(ctx, cfg, dH[m], st, need, out=outs[0] if m == "text" else outs[1])
    return dX.get("text"), dX.get("image"), dE.get("text"), dE.get("image")
