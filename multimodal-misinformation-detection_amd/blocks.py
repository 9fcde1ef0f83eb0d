"""Forward/backward building blocks shared by the fusion head and the encoders.

Every function here only sequences kernel launches (kernels.py); there is no torch math. A
`StepCtx` carries the per-call policy: activation dtype (fp32 parity mode / bf16 throughput mode),
dropout probability and the device-resident step seed, the weight views in compute dtype and the
parameter-gradient accumulators (first write overwrites, later writes accumulate with beta=1, so
tensors used by several paths — the shared MLPs / Q projections of model.py:165-166,188-228 — sum
their gradients inside the GEMM epilogue).
"""
from __future__ import annotations

import os
import weakref

import torch

from . import kernels as K

_SIDE = {}


def side_stream(device):
    """Per-device stream for the weight-gradient GEMMs: they only depend on tensors the main
    stream already produced, and nothing on the main stream reads their outputs until the layer's
    gradients are reported (join), so they overlap with the data-gradient chain (dX GEMMs,
    attention and LayerNorm backward). Opt-in (MMFD_SIDE_STREAM=1): with one 256x256 GEMM block
    per CU the two streams only partition the CUs, and no gain was measured (1734 vs 1730 pairs/s)."""
    if os.environ.get("MMFD_SIDE_STREAM", "0") != "1" or device.type != "cuda":
        return None
    s = _SIDE.get(device.index)
    if s is None:
        s = _SIDE[device.index] = torch.cuda.Stream(device=device)
    return s


# Persistent compute-dtype copies of the fp32 master weights ("shadows"). A module keeps its
# shadows across steps (`shadow_store(module)`: key -> (bf16 tensor, [(param name, data_ptr,
# version)])); SHADOW_OF maps a master parameter's data_ptr to the bf16 view that mmfd.optim.AdamW
# refreshes in the same kernel that updates the parameter (mmfd_adamw's param_bf16), so the
# weights are cast once, not once per step. Any other in-place update of a parameter (load_state_dict,
# torch optimizers, manual edits) bumps its version counter, and the shadow is re-cast.
# Entries: data_ptr -> (bf16 view, (id(store), key), weakref(store)). When a module dies its store's
# finalizer drops its entries (the bf16 copies are freed with it), and live_shadow() ignores any
# entry whose store is gone — the allocator hands the pointers to the next model's weights, which must
# get shadows of their own instead of AdamW writing into a dead model's copies.
SHADOW_OF = {}


class _ShadowStore(dict):
    """a module's shadow store (a dict that SHADOW_OF can hold weakly)"""


def live_shadow(ptr):
    """SHADOW_OF[ptr] if its owning store is still alive, else None (and the stale entry is removed)"""
    e = SHADOW_OF.get(ptr)
    if e is not None and e[2]() is None:
        del SHADOW_OF[ptr]
        return None
    return e


def _drop_dead_store(sid):
    """a store's finalizer: its SHADOW_OF entries go with it (the bf16 copies are freed with the module)"""
    for ptr in [k for k, v in SHADOW_OF.items() if v[1][0] == sid and v[2]() is None]:
        del SHADOW_OF[ptr]


def shadow_store(module):
    st = module.__dict__.get("_mmfd_shadows")
    if st is None:
        st = module.__dict__["_mmfd_shadows"] = _ShadowStore()
        weakref.finalize(st, _drop_dead_store, id(st))
    return st


def invalidate_caches(module):
    """Drop every weight-derived tensor of `module` (compute-dtype shadows, packed biases, position-
    bias tables): the next forward rebuilds them from the master parameters. Needed after writes
    that bypass torch's version counter (`p.data.copy_(...)`, `p.data[...] = ...`);
    load_state_dict / .to() / .cuda() call it themselves (CachedWeights)."""
    st = module.__dict__.get("_mmfd_shadows")
    if st:
        sid = id(st)
        for ptr in [k for k, v in SHADOW_OF.items() if v[1][0] == sid]:
            del SHADOW_OF[ptr]
        st.clear()


class CachedWeights:
    """Mixin for nn.Modules that keep weight-derived caches (shadow_store): invalidated by
    load_state_dict and by _apply (.to / .cuda / .float ...), and on demand by invalidate_caches()."""

    def invalidate_caches(self):
        invalidate_caches(self)
        return self

    def load_state_dict(self, *a, **kw):
        r = super().load_state_dict(*a, **kw)
        invalidate_caches(self)
        return r

    def _apply(self, *a, **kw):
        r = super()._apply(*a, **kw)
        invalidate_caches(self)
        return r


ATTN_DROP_MASK = os.environ.get("MMFD_ATTN_DROP_MASK") == "1"


class StepCtx:
    def __init__(self, params: dict, dtype: torch.dtype, dropout_p: float = 0.0, seed: K.Seed | None = None,
                 training: bool = False, shadows: dict | None = None):
        self.P = params          # name -> fp32 master tensor (nn.Parameter data)
        self.shadows = shadows   # persistent shadow store of the owning module (see SHADOW_OF)
        self.dt = dtype
        self.p = float(dropout_p) if training else 0.0
        self.seed = seed
        self.training = training
        self._w = {}             # cached compute-dtype weights
        self.grads = {}          # name -> fp32 grad tensor
        self._written = set()
        self.grad_ready = None   # optional callable(names, grads): finished gradients (DP overlap)
        self._notified = set()
        self.side = None         # stream for weight-gradient GEMMs (enable_side_stream)
        self.cache_derived = False  # keep weight-derived tensors across calls (see derived())
        self._side_used = False
        self._wp = {}            # split planes of fp32 weights, by data_ptr (one split per call)
        self._dmask = {}         # attention site -> dropout keep-bitmask (forward writes, backward reads)

    def enable_side_stream(self, device):
        self.side = side_stream(device)
        return self

    def join_side(self):
        """main stream waits for every weight-gradient GEMM issued so far"""
        if self.side is not None and self._side_used:
            torch.cuda.current_stream().wait_stream(self.side)
            self._side_used = False

    # ---- weights -------------------------------------------------------------------------------
    def _shadow(self, key, pnames):
        """the persistent compute-dtype copy of the row-concatenated weights `pnames`, or None when
        it has to be (re)built (absent, a master weight changed outside mmfd's AdamW, or a weight
        already shadowed under another key)"""
        if self.shadows is None:
            return None
        ent = self.shadows.get(key)
        if ent is None:
            return None
        t, members = ent
        for n, ptr, ver in members:
            src = self.P[n]
            if src.data_ptr() != ptr or src._version != ver or live_shadow(ptr) is None:
                return None
        return t

    def _register(self, key, t, pnames):
        """record `t` (rows of the weights `pnames`) as their shadow when none of them has one yet"""
        if self.shadows is None:
            return
        r, members, views = 0, [], []
        for n in pnames:
            src = self.P[n]
            ptr = src.data_ptr()
            owner = live_shadow(ptr)
            if owner is not None and owner[1] != (id(self.shadows), key):
                return  # shadowed elsewhere: this key is re-cast every step
            views.append((ptr, t[r:r + src.shape[0]]))
            members.append((n, ptr, src._version))
            r += src.shape[0]
        ref = weakref.ref(self.shadows) if isinstance(self.shadows, _ShadowStore) else (lambda: self.shadows)
        for ptr, v in views:
            SHADOW_OF[ptr] = (v, (id(self.shadows), key), ref)
        self.shadows[key] = (t, members)

    def w(self, name):
        """weight `name.weight` in compute dtype"""
        key = name
        t = self._w.get(key)
        if t is None:
            src = self.P[name + ".weight"]
            if self.dt == torch.float32:
                t = src
            else:
                t = self._shadow(key, [name + ".weight"])
                if t is None:
                    t = K.cast(src, self.dt)
                    self._register(key, t, [name + ".weight"])
            self._w[key] = t
        return t

    def wT(self, name):
        """the K-contiguous copy W^T [in, out] of weight `name.weight` in compute dtype (mmfd_transpose
        of the shadow, made once per step: the data-gradient GEMM dY W then runs in the forward
        operand layout, on the four-wave kernel)"""
        key = name + "^T"
        t = self._w.get(key)
        if t is None:
            t = self._w[key] = K.transpose(self.w(name))
        return t

    def b(self, name):
        return self.P.get(name + ".bias")

    def w_packed(self, names):
        """row-concatenation of several nn.Linear weights (fused QKV / K|V GEMM) in compute dtype"""
        key = "|".join(names)
        t = self._w.get(key)
        if t is None:
            wn = [n + ".weight" for n in names]
            ws = [self.P[n] for n in wn]
            rows = sum(w.shape[0] for w in ws)
            t = self._shadow(key, wn) if self.dt != torch.float32 else None
            if t is None:
                t = torch.empty((rows, ws[0].shape[1]), device=ws[0].device, dtype=self.dt)
                r = 0
                for w in ws:
                    K.cast(w, self.dt, out=t[r:r + w.shape[0]])
                    r += w.shape[0]
                if self.dt != torch.float32:
                    self._register(key, t, wn)
            def pack_bias():
                bt = torch.empty(rows, device=ws[0].device, dtype=torch.float32)
                r = 0
                for n, w in zip(names, ws):
                    bb = self.P.get(n + ".bias")
                    if bb is None:   # bias-free projection (Swinv2 key): zero slice of the packed bias
                        bt[r:r + w.shape[0]].zero_()
                    else:
                        K.cast(bb, torch.float32, out=bt[r:r + bb.shape[0]])
                    r += w.shape[0]
                return bt
            self._w[key] = t
            self._w[key + "#bias"] = self.derived(key + "#bias", [n + ".bias" for n in names if n + ".bias" in self.P],
                                                  pack_bias)
        return t, self._w[key + "#bias"]

    def derived(self, key, pnames, make):
        """a tensor computed from the parameters `pnames` only (packed biases, Swinv2 position-bias
        tables), kept in the module's persistent store and rebuilt when any of them changed
        (data pointer or version counter), and dropped by invalidate_caches() / load_state_dict.
        Opt-in per context (`cache_derived`): only for frozen, inference-only encoders — mmfd's
        AdamW writes parameters through raw pointers without bumping torch's version counter, so
        training contexts always rebuild."""
        if self.shadows is None or not self.cache_derived:
            return make()
        sig = tuple((self.P[n].data_ptr(), self.P[n]._version) for n in pnames)
        ent = self.shadows.get(("derived", key))
        if ent is not None and ent[0] == sig:
            return ent[1]
        t = make()
        self.shadows[("derived", key)] = (sig, t)
        return t

    def wplanes(self, W):
        """split planes of an fp32 weight matrix, made once per forward/backward of the module and
        shared by its forward and data-gradient GEMMs (None outside split-operand fp32 mode)"""
        if self.dt != torch.float32 or not K.split_eligible(W):
            return None
        key = (W.data_ptr(), tuple(W.shape), W.stride(0))
        p = self._wp.get(key)
        if p is None:
            p = self._wp[key] = K.split3(W)
        return p

    def planes(self, t):
        """bf16 planes of an fp32 GEMM operand (kernels.split3) when the fp32 GEMMs run on split
        operands, else None: split once, read by every GEMM that takes `t` (the forward input
        again by its weight-gradient GEMM, an output gradient by the data- and weight-gradient
        GEMMs) instead of being split inside each of them"""
        if self.dt != torch.float32 or not K.split_eligible(t):
            return None
        return K.split3(t)

    # ---- dropout -------------------------------------------------------------------------------
    def drop(self, site):
        """(p, seed, salt) kwargs for a dropout site; p=0 when not training."""
        if self.p <= 0.0:
            return {}
        return dict(dropout_p=self.p, seed=self.seed, salt=K.salt_of(site))

    def attn_drop(self, site, q=None, k=None, H=None):
        """dropout kwargs of an attention call, plus — with MMFD_ATTN_DROP_MASK=1 — its keep-bitmask:
        the forward call (q, k, H given) allocates the mask the kernel writes, the backward call of
        the same site passes the same buffer and reads it instead of re-hashing. Off by default:
        measured slower (tools/attn_bench.py, round 4: BERT fp32 fwd 369 -> 390 us, bwd 986 -> 996
        us; bf16 162 -> 169 / 441 -> 444 us) — the backward kernels are not bound by the hash."""
        kw = self.drop(site)
        if not kw or not ATTN_DROP_MASK:
            return kw
        if q is not None:
            self._dmask[site] = K.drop_mask_buffer(q.shape[0], H, q.shape[1], k.shape[1], q.device)
        m = self._dmask.get(site)
        return dict(kw, drop_mask=m) if m is not None else kw

    # ---- gradients -----------------------------------------------------------------------------
    def flush_ready(self):
        """report the gradients written since the last call as final (a layer's backward is done)"""
        if self.grad_ready is None:
            return
        self.join_side()
        names = [n for n in self.grads if n not in self._notified]
        if names:
            self._notified.update(names)
            self.grad_ready(names, self.grads)

    def grad_slot(self, pname, shape):
        """(tensor, beta) for accumulating into the gradient of parameter `pname`."""
        g = self.grads.get(pname)
        if g is None:
            g = torch.empty(shape, device=self.P[pname].device, dtype=torch.float32)
            self.grads[pname] = g
            return g, 0.0
        return g, 1.0

    def lin_grads(self, names, dy2d, x2d, dyp=None, xp=None):
        if self.side is None:
            return self._lin_grads(names, dy2d, x2d, dyp, xp)
        self.side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(self.side):
            self._lin_grads(names, dy2d, x2d, dyp, xp)
        for t in (dy2d, x2d, dyp, xp):
            if t is not None:
                t.record_stream(self.side)
        self._side_used = True

    def _lin_grads(self, names, dy2d, x2d, dyp=None, xp=None):
        """dW = dy^T x (fp32, accumulate) with db = sum_rows(dy) fused into the same GEMM
        (a_rowsum); `names` are the row blocks of dy. A packed group (fused QKV / K|V) whose
        gradients are first written here is ONE GEMM into a packed buffer whose row blocks become
        the parameters' gradient tensors."""
        fresh = all(n + ".weight" not in self.grads and n + ".bias" not in self.grads for n in names)
        has_b = all(n + ".bias" in self.P for n in names)
        if len(names) > 1 and fresh and has_b:
            rows = [self.P[n + ".weight"].shape[0] for n in names]
            kin = self.P[names[0] + ".weight"].shape[1]
            dev = self.P[names[0] + ".weight"].device
            gw = torch.empty((sum(rows), kin), device=dev, dtype=torch.float32)
            gb = torch.empty(sum(rows), device=dev, dtype=torch.float32)
            K.gemm(dy2d, x2d, trans_a=True, trans_b=True, out=gw, a_rowsum=gb, a_planes=dyp, b_planes=xp)
            r = 0
            for n, k in zip(names, rows):
                self.grads[n + ".weight"] = gw[r:r + k]
                self.grads[n + ".bias"] = gb[r:r + k]
                r += k
            return
        if len(names) == 1:
            n = names[0]
            g, beta = self.grad_slot(n + ".weight", self.P[n + ".weight"].shape)
            if n + ".bias" in self.P:
                gb, bb = self.grad_slot(n + ".bias", self.P[n + ".bias"].shape)
                K.gemm(dy2d, x2d, trans_a=True, trans_b=True, out=g, beta=beta, a_rowsum=gb, a_rowsum_beta=bb,
                       a_planes=dyp, b_planes=xp)
            else:
                K.gemm(dy2d, x2d, trans_a=True, trans_b=True, out=g, beta=beta, a_planes=dyp, b_planes=xp)
            return
        r = 0
        for n in names:
            rows = self.P[n + ".weight"].shape[0]
            # (a planes-only gradient has no fp32 copy to slice: slice its planes instead)
            dys = dy2d[:, r:r + rows]
            if getattr(dy2d, "_mmfd_planes_only", False):
                dys._mmfd_planes_only = True
            self._lin_grads([n], dys, x2d, dyp[:, :, r:r + rows].contiguous() if dyp is not None else None, xp)
            r += rows


def as2d(x):
    return x.reshape(-1, x.shape[-1])


# -------------------------------------------------------------------------------------------------
# linear
# -------------------------------------------------------------------------------------------------
# the training forward's GELU keeps gelu'(pre-activation) instead of the pre-activation
# (MMFD_ACT_GELU_D; one erf per element instead of one in the forward and one in the backward) when a
# kernel with it in its own epilogue runs the product (bf16: the four-wave GEMM; fp32: the
# split-operand GEMM's ext instantiation); MMFD_GELU_DERIV=0 keeps the pre-activation (A/B switch)
GELU_DERIV = os.environ.get("MMFD_GELU_DERIV", "1") != "0"


def linear(ctx: StepCtx, x2d, name, *, act=K.ACT_NONE, keep_aux=False, residual=None, drop_site=None,
           out_dtype=None, xp=None, out_planes=None, write_out=True):
    """(y, aux): with keep_aux, aux is what the activation's backward reads — the pre-activation,
    or for GELU under GELU_DERIV its derivative (tagged _mmfd_gelu_d; linear_dx then multiplies)"""
    W = ctx.w(name)
    aux = None
    if keep_aux and act in (K.ACT_GELU, K.ACT_RELU):
        aux = torch.empty((x2d.shape[0], W.shape[0]), device=x2d.device, dtype=out_dtype or ctx.dt)
        # (bf16: the four-wave kernel's register epilogue; fp32: the split-operand kernel's ext
        # instantiation — planes of x given means the product runs on split operands)
        if act == K.ACT_GELU and GELU_DERIV and residual is None and drop_site is None and (
                K.g4_takes(x2d, W, act) or (ctx.dt == torch.float32 and xp is not None)):
            act = K.ACT_GELU_D
            aux._mmfd_gelu_d = True
    y = K.gemm(x2d, W, bias=ctx.b(name), act=act, aux=aux, residual=residual, out_dtype=out_dtype or ctx.dt,
               a_planes=xp, b_planes=ctx.wplanes(W) if xp is not None else None, out_planes=out_planes,
               write_out=write_out, **(ctx.drop(drop_site) if drop_site else {}))
    return y, aux


def new_planes(ctx: StepCtx, rows, cols, device):
    """an empty bf16 [3, rows, cols] planes buffer for a producer kernel to fill in split-operand fp32
    mode, else None"""
    if ctx.dt != torch.float32 or K.fp32_gemm_mode() != 1 or cols % 8 or 6 * rows * cols >= (1 << 31) - 4096:
        return None
    return torch.empty((3, rows, cols), device=device, dtype=torch.bfloat16)


def out_planes(ctx: StepCtx, rows, cols, consumers, device):
    """(planes, write_out) for a GEMM output in split-operand fp32 mode: bf16 [3, rows, cols]
    written by the producing epilogue, and whether the fp32 output is needed at all — it is not
    when every consumer GEMM ((M, N, K, trans_a, trans_b) tuples) runs on split operands.
    (None, True) otherwise."""
    if ctx.dt != torch.float32 or K.fp32_gemm_mode() != 1 or cols % 8 or os.environ.get("MMFD_NO_EPI_PLANES"):
        return None, True
    pl = torch.empty((3, rows, cols), device=device, dtype=torch.bfloat16)
    return pl, not all(K.x6_ok(*c) for c in consumers)


def linear_packed(ctx: StepCtx, x2d, names, xp=None):
    W, b = ctx.w_packed(names)
    return K.gemm(x2d, W, bias=b, a_planes=xp, b_planes=ctx.wplanes(W) if xp is not None else None)


# A/B switch (same-box bench comparisons): 0 = never, 2 = also past the four-wave kernel's K limit
# (those products then run on gemm256_kernel in the forward layout)
DX_TRANSPOSED = os.environ.get("MMFD_DX_TRANSPOSED", "1")


def _dx_forward_layout(ctx, dy2d, name_or_W, out, beta, act, residual, drop_site):
    """whether dY W runs better as dY (W^T)^T with the transposed weight copy: bf16 products the
    four-wave GEMM takes in the forward layout (K = out features <= its K limit, full 256x256
    tiles; a plain, + residual or GELU-backward epilogue) — the FFN2 and attention-output data
    gradients"""
    if DX_TRANSPOSED == "0" or ctx.dt != torch.bfloat16 or not isinstance(name_or_W, str) or out is not None:
        return False
    if beta != 0.0:
        return False
    if drop_site is not None or act not in (K.ACT_NONE, K.ACT_GELU_BWD, K.ACT_MUL_AUX) or (residual is not None and act != K.ACT_NONE):
        return False
    mode, kmax = K.g4_mode()
    if mode == "off":
        return False
    nout, nin = ctx.P[name_or_W + ".weight"].shape
    if DX_TRANSPOSED == "2":
        kmax = 1 << 30
    return dy2d.shape[0] % 256 == 0 and nin % 256 == 0 and nout % 64 == 0 and 64 <= nout <= kmax


def linear_dx(ctx: StepCtx, dy2d, name_or_W, *, out=None, beta=0.0, act=K.ACT_NONE, aux=None, drop_site=None,
              residual=None, dyp=None, out_planes=None, write_out=True):
    if act == K.ACT_GELU_BWD and getattr(aux, "_mmfd_gelu_d", False):
        act = K.ACT_MUL_AUX  # aux already holds gelu'(pre-activation)
    if _dx_forward_layout(ctx, dy2d, name_or_W, out, beta, act, residual, drop_site):
        return K.gemm(dy2d, ctx.wT(name_or_W), act=act, aux=aux, residual=residual)
    W = ctx.w(name_or_W) if isinstance(name_or_W, str) else name_or_W
    return K.gemm(dy2d, W, trans_b=True, out=out, beta=beta if out is not None else 0.0, act=act, aux=aux,
                  residual=residual, a_planes=dyp, b_planes=ctx.wplanes(W) if dyp is not None else None,
                  out_planes=out_planes, write_out=write_out,
                  **(ctx.drop(drop_site) if drop_site else {}))


# -------------------------------------------------------------------------------------------------
# LayerNorm
# -------------------------------------------------------------------------------------------------
def layernorm(ctx: StepCtx, x2d, name, eps):
    return K.layernorm_fwd(x2d, ctx.P[name + ".weight"], ctx.P[name + ".bias"], eps)


# ablation switch: MMFD_NO_LN_PLANES=1 splits LayerNorm outputs in separate passes (split3) instead
_NO_LN_PLANES = os.environ.get("MMFD_NO_LN_PLANES") == "1"


def layernorm_planes(ctx: StepCtx, x2d, name, eps, want=True):
    """(y, mean, rstd, planes): the LayerNorm output and, when `want` and the fp32 GEMMs run on split
    operands, its split planes written by the same kernel (else None)"""
    if want and ctx.dt == torch.float32 and x2d.shape[1] % 8 == 0 and K.split_eligible(x2d) and not _NO_LN_PLANES:
        pl = torch.empty((3, x2d.shape[0], x2d.shape[1]), device=x2d.device, dtype=torch.bfloat16)
        y, m, r = K.layernorm_fwd(x2d, ctx.P[name + ".weight"], ctx.P[name + ".bias"], eps, planes=pl)
        return y, m, r, pl
    y, m, r = layernorm(ctx, x2d, name, eps)
    return y, m, r, None


def layernorm_bwd_planes(ctx: StepCtx, dy2d, x2d, name, mean, rstd, *, dx_add=None, drop_site=None):
    """layernorm_bwd plus the split planes of the gradient the next GEMMs read (the dropped one when
    there is dropout), written by the same kernel in split-operand fp32 mode (else None):
    (dx, dx_dropped or None, planes or None)"""
    W = dy2d.shape[1]
    if not (ctx.dt == torch.float32 and W % 8 == 0 and W // 4 > 32 and K.split_eligible(dy2d)) or _NO_LN_PLANES:
        dx, dd = layernorm_bwd(ctx, dy2d, x2d, name, mean, rstd, dx_add=dx_add, drop_site=drop_site)
        return dx, dd, None
    pl = torch.empty((3, dy2d.shape[0], W), device=dy2d.device, dtype=torch.bfloat16)
    dx, dd = layernorm_bwd(ctx, dy2d, x2d, name, mean, rstd, dx_add=dx_add, drop_site=drop_site, planes=pl)
    return dx, dd, pl


def layernorm_bwd(ctx: StepCtx, dy2d, x2d, name, mean, rstd, *, dx_add=None, drop_site=None, planes=None):
    """Returns (dx, dx_dropped or None). Gamma/beta grads accumulate into ctx.grads."""
    gw, bw = ctx.grad_slot(name + ".weight", ctx.P[name + ".weight"].shape)
    gb, bb = ctx.grad_slot(name + ".bias", ctx.P[name + ".bias"].shape)
    assert bw == bb
    dd = None
    kw = {}
    if drop_site is not None and ctx.p > 0:
        dd = torch.empty_like(dy2d)
        kw = dict(dx_drop=dd, dropout_p=ctx.p, seed=ctx.seed, salt=K.salt_of(drop_site))
    dx = K.layernorm_bwd(dy2d, x2d, ctx.P[name + ".weight"], mean, rstd, dx_add=dx_add, dgamma=gw, dbeta=gb,
                         beta_acc=bw, planes=planes, **kw)
    return dx, dd


# -------------------------------------------------------------------------------------------------
# MLP block:  y = LN(a + drop(W2 drop(gelu(W1 a + b1)) + b2))     (layers.py:12-18 + model.py:109)
# -------------------------------------------------------------------------------------------------
def mlp_ln_fwd(ctx: StepCtx, a2d, mlp, ln, site, eps=1e-5, w1=".net.0", w2=".net.3", ap=None, want_planes=False):
    """`ap`: split planes of a2d (split-operand fp32 mode, else None); the hidden activation's planes
    come from the W1 epilogue (no fp32 copy when both of its GEMMs run on split operands), and with
    `want_planes` the LayerNorm also writes the output's planes. Returns (y, yp or None, state)."""
    T, E = a2d.shape
    I = ctx.P[mlp + w1 + ".weight"].shape[0]
    hp, h_out = out_planes(ctx, T, I, [(T, E, I), (E, I, T, True, True)], a2d.device) if ap is not None \
        else (None, True)
    h, pre = linear(ctx, a2d, mlp + w1, act=K.ACT_GELU, keep_aux=True, drop_site=site + ".h", xp=ap, out_planes=hp,
                    write_out=h_out)
    s, _ = linear(ctx, h, mlp + w2, residual=a2d, drop_site=site + ".out", xp=hp)
    y, mean, rstd, yp = layernorm_planes(ctx, s, ln, eps, want=want_planes)
    return y, yp, (a2d, ap, h, hp, pre, s, mean, rstd, mlp, ln, site, w1, w2)


def mlp_ln_bwd(ctx: StepCtx, dy2d, st):
    a2d, ap, h, hp, pre, s, mean, rstd, mlp, ln, site, w1, w2 = st
    ds, ds_drop, gp = layernorm_bwd_planes(ctx, dy2d, s, ln, mean, rstd, drop_site=site + ".out") \
        if ap is not None else (*layernorm_bwd(ctx, dy2d, s, ln, mean, rstd, drop_site=site + ".out"), None)
    g_out = ds_drop if ds_drop is not None else ds
    ctx.lin_grads([mlp + w2], g_out, h, gp, hp)
    T, E = g_out.shape
    I = h.shape[1]
    dprep, dpre_out = out_planes(ctx, T, I, [(I, E, T, True, True), (T, E, I, False, True)], g_out.device) \
        if gp is not None else (None, True)
    dpre = linear_dx(ctx, g_out, mlp + w2, act=K.ACT_GELU_BWD, aux=pre, drop_site=site + ".h", dyp=gp,
                     out_planes=dprep, write_out=dpre_out)
    ctx.lin_grads([mlp + w1], dpre, a2d, dprep, ap)
    linear_dx(ctx, dpre, mlp + w1, out=ds, beta=1.0, dyp=dprep)  # da = ds + dpre W1
    return ds


def load_state_dict_checked(module, state_dict, benign=("position_ids", "num_batches_tracked")):
    """module.load_state_dict(strict=False) that fails like strict loading on every missing or
    unexpected key except the named benign ones (matched as a key suffix or a "prefix." start): a
    checkpoint whose names do not match must not leave random weights behind plausible outputs"""
    res = module.load_state_dict(state_dict, strict=False)
    ok = lambda k: any(k.endswith(b) or k.startswith(b + ".") for b in benign)  # noqa: E731
    missing = [k for k in res.missing_keys if not ok(k)]
    unexpected = [k for k in res.unexpected_keys if not ok(k)]
    if missing or unexpected:
        raise RuntimeError(f"{type(module).__name__}: state_dict does not match: missing {missing[:8]}"
                           f"{' ...' if len(missing) > 8 else ''}, unexpected {unexpected[:8]}"
                           f"{' ...' if len(unexpected) > 8 else ''}")
    return res
