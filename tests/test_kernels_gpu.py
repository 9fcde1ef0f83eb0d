"""Kernel-level numerics of libmmfd_hip.so against plain PyTorch fp64/fp32 references (CPU).

Tolerances: fp32 kernels accumulate in fp32 on MFMA (exact fp32 products) -> rel 2e-5 of the
operand scale; bf16 kernels round inputs/outputs to bf16 (8 significant bits) -> rel 2e-2.
"""
import math

import numpy as np
import pytest
import torch

import mmfd
from mmfd import kernels as K
from oracle.dropout_hash import attn_keep_mask, keep_mask

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _tol(dtype):
    return (3e-5, 3e-5) if dtype == torch.float32 else (2e-2, 2e-2)


def _close(got, ref, dtype, scale=1.0):
    rtol, atol = _tol(dtype)
    got = got.detach().double().cpu()
    ref = ref.detach().double().cpu()
    err = (got - ref).abs().max().item()
    bound = atol * scale + rtol * ref.abs().max().item()
    assert err <= bound, f"max err {err:.3e} > {bound:.3e}"


def _rand(*shape, dtype=torch.float32, scale=1.0, seed=0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(dtype)


# ---------------------------------------------------------------------------------------------
# GEMM
# ---------------------------------------------------------------------------------------------
SHAPES = [(128, 128, 64), (256, 384, 768), (200, 136, 96), (37, 24, 40), (1000, 256, 512), (64, 3072, 768)]


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("layout", ["nt", "nn", "tn"])
@pytest.mark.parametrize("shape", SHAPES)
def test_gemm_layouts(dtype, layout, shape):
    M, N, Kd = shape
    if layout == "nt":  # y = x W^T
        A = _rand(M, Kd, dtype=dtype, seed=1); B = _rand(N, Kd, dtype=dtype, seed=2)
        ref = A.double() @ B.double().T
        out = K.gemm(A.to(DEV), B.to(DEV), out_dtype=torch.float32)
    elif layout == "nn":  # dX = dY W
        A = _rand(M, Kd, dtype=dtype, seed=1); B = _rand(Kd, N, dtype=dtype, seed=2)
        ref = A.double() @ B.double()
        out = K.gemm(A.to(DEV), B.to(DEV), trans_b=True, out_dtype=torch.float32)
    else:  # dW = dY^T X
        A = _rand(Kd, M, dtype=dtype, seed=1); B = _rand(Kd, N, dtype=dtype, seed=2)
        ref = A.double().T @ B.double()
        out = K.gemm(A.to(DEV), B.to(DEV), trans_a=True, trans_b=True, out_dtype=torch.float32)
    torch.cuda.synchronize()
    rtol = 2e-5 if dtype == torch.float32 else 2e-5  # inputs exact in both; fp32 accumulation
    err = (out.double().cpu() - ref).abs().max().item()
    assert err <= rtol * math.sqrt(Kd) * 4 + 1e-4, err


@pytest.mark.parametrize("layout", ["nt", "nn", "tn", "tt"])
@pytest.mark.parametrize("Kd", [64, 128, 192, 256, 320])
def test_gemm_bf16_g8_ktile_counts(layout, Kd):
    """the bf16 G8 loop at 1-5 K-tiles (round 5: each phase's kc = 0 fragments are read one phase
    ahead, with counted waits that change at the last two K-tiles), every operand layout, ragged
    M / N, fp32 and bf16 outputs, against fp64"""
    M, N = 300, 520
    ta, tb = layout[0] == "t", layout[1] == "t"
    A = _rand(*((Kd, M) if ta else (M, Kd)), dtype=torch.bfloat16, seed=Kd + 1)
    B = _rand(*((Kd, N) if tb else (N, Kd)), dtype=torch.bfloat16, seed=Kd + 2)
    ref = (A.double().T if ta else A.double()) @ (B.double() if tb else B.double().T)
    for odt in (torch.float32, torch.bfloat16):
        out = K.gemm(A.to(DEV), B.to(DEV), trans_a=ta, trans_b=tb, out_dtype=odt)
        torch.cuda.synchronize()
        err = (out.double().cpu() - ref).abs().max().item() / ref.abs().max().item()
        assert err <= (1e-5 if odt == torch.float32 else 8e-3), (odt, err)


@pytest.fixture
def g4_restore():
    """the four-wave GEMM switches (mmfd_set_g4_mode / _kmax) as they were before the test"""
    old, persist = K.g4_mode(), K.set_g4_persist()
    yield
    K.set_g4_mode(*old)
    K.set_g4_persist(persist)


@pytest.mark.parametrize("shape", [(256, 256, 64), (512, 768, 128), (768, 2304, 768), (1024, 512, 1024),
                                   (2048, 3072, 768)])
@pytest.mark.parametrize("with_bias", [False, True])
def test_gemm_bf16_g4_forward(shape, with_bias, g4_restore):
    """the four-wave assembly-scheduled forward GEMM (gemm_g4.hip: bf16 -> bf16, K-contiguous
    operands, full 256x256 tiles, bias epilogue) against fp64, and against gemm256_kernel on the same
    inputs (MMFD_G4=0 routes the product there): both accumulate each output's K in the same order
    of 16x16x32 MFMAs from zero and round once to bf16"""
    M, N, Kd = shape
    A = _rand(M, Kd, dtype=torch.bfloat16, seed=M + 7).to(DEV)
    B = _rand(N, Kd, dtype=torch.bfloat16, seed=N + 8).to(DEV)
    bias = _rand(N, seed=Kd + 9).to(DEV) if with_bias else None
    ref = A.double().cpu() @ B.double().cpu().T + (bias.double().cpu() if with_bias else 0.0)
    K.set_g4_mode("on")
    g4 = K.gemm(A, B, bias=bias)
    K.set_g4_mode("off")
    g8 = K.gemm(A, B, bias=bias)
    torch.cuda.synchronize()
    err = (g4.double().cpu() - ref).abs().max().item() / ref.abs().max().item()
    assert err <= 8e-3, err
    diff = (g4.float() - g8.float()).abs().max().item()
    ulp = (g8.float().abs().max().item() * 2.0 ** -7)
    assert diff <= ulp, (diff, ulp)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", [(768, 3072), (3072, 768), (77, 130), (1, 64), (300, 1)])
def test_transpose_exact(shape, dtype):
    """mmfd_transpose (the per-step K-contiguous weight copy): exact, odd shapes and a strided view"""
    x = _rand(*shape, dtype=dtype, seed=shape[0] + shape[1]).to(DEV)
    assert torch.equal(K.transpose(x), x.t().contiguous())
    wide = _rand(shape[0], shape[1] + 8, dtype=dtype, seed=5).to(DEV)
    v = wide[:, 8:]
    assert torch.equal(K.transpose(v), v.t().contiguous())


@pytest.mark.parametrize("act", ["none", "gelu_bwd", "mul_aux"])
@pytest.mark.parametrize("shape", [(512, 3072, 768), (768, 768, 768), (256, 256, 64)])
def test_gemm_bf16_dx_forward_layout_matches_trans_b(shape, act, g4_restore):
    """the bf16 data-gradient GEMM dY W run as dY (W^T)^T on the four-wave kernel (blocks.linear_dx
    with the transposed weight copy; EPI 4 = x GELU'(pre-activation)) gives the same bits as the
    product with W as the MN-contiguous operand on gemm256_kernel"""
    M, N, Kd = shape  # dY [M, Kd] (out features), W [Kd, N] (nn.Linear [out, in])
    dy = _rand(M, Kd, dtype=torch.bfloat16, seed=M + 1).to(DEV)
    W = _rand(Kd, N, dtype=torch.bfloat16, seed=N + 2).to(DEV)
    kw = {}
    if act == "gelu_bwd":
        kw = dict(act=K.ACT_GELU_BWD, aux=_rand(M, N, dtype=torch.bfloat16, seed=3).to(DEV))
    elif act == "mul_aux":  # EPI 6: x the saved GELU derivative
        kw = dict(act=K.ACT_MUL_AUX, aux=_rand(M, N, dtype=torch.bfloat16, seed=3).to(DEV))
    K.set_g4_mode("on")
    g4 = K.gemm(dy, K.transpose(W), **kw)
    ref = K.gemm(dy, W, trans_b=True, **kw)
    K.set_g4_mode("off")
    g8 = K.gemm(dy, K.transpose(W), **kw)
    torch.cuda.synchronize()
    assert torch.equal(g4, g8), (g4.float() - g8.float()).abs().max().item()
    assert torch.equal(g4, ref), (g4.float() - ref.float()).abs().max().item()


@pytest.mark.parametrize("Kd", [64, 768])
@pytest.mark.parametrize("mode", ["bias", "gelu_aux", "dropout_residual"])
def test_gemm_bf16_g4_strided_views_match_g8(Kd, mode, g4_restore):
    """the four-wave kernel on column-sliced views — lda / ldb > K (a Q|K|V slice of a
    packed activation), ldc / ldr / ldaux > N — is bit-identical to gemm256_kernel, K = 64 (one K-tile:
    the two-tile-ahead prefetch reads past K inside the row's buffer range) included; the bytes of
    the wider buffers outside the views stay untouched"""
    M, N = 512, 768
    A_full = _rand(M, Kd + 128, dtype=torch.bfloat16, seed=61).to(DEV)
    B_full = _rand(N, Kd + 64, dtype=torch.bfloat16, seed=62).to(DEV)
    A, B = A_full[:, 64:64 + Kd], B_full[:, 32:32 + Kd]  # 16-B aligned column slices
    bias = _rand(N, seed=63).to(DEV)
    res_full = _rand(M, N + 256, dtype=torch.bfloat16, seed=64).to(DEV)
    res = res_full[:, 128:128 + N]
    outs = {}
    for g4 in ("1", "0"):
        K.set_g4_mode("gelu" if g4 == "1" else "off")
        c_full = torch.full((M, N + 512), 3.0, dtype=torch.bfloat16, device=DEV)
        x_full = torch.full((M, N + 128), 5.0, dtype=torch.bfloat16, device=DEV)
        c, x = c_full[:, 256:256 + N], x_full[:, 64:64 + N]
        if mode == "bias":
            K.gemm(A, B, bias=bias, out=c)
        elif mode == "gelu_aux":
            K.gemm(A, B, bias=bias, act=K.ACT_GELU, aux=x, out=c)
        else:
            K.gemm(A, B, bias=bias, residual=res, dropout_p=0.1, seed=K.Seed(78, device=DEV), salt=6, out=c)
        outs[g4] = (c_full, x_full)
    torch.cuda.synchronize()
    assert torch.equal(outs["1"][0], outs["0"][0])
    assert torch.equal(outs["1"][1], outs["0"][1])
    c_full, x_full = outs["1"]
    assert bool((c_full[:, :256] == 3.0).all()) and bool((c_full[:, 256 + N:] == 3.0).all())
    if mode == "gelu_aux":
        assert bool((x_full[:, :64] == 5.0).all()) and bool((x_full[:, 64 + N:] == 5.0).all())
    ref = A.double().cpu() @ B.double().cpu().T + bias.double().cpu()
    got = outs["1"][1][:, 64:64 + N] if mode == "gelu_aux" else outs["1"][0][:, 256:256 + N]
    if mode != "dropout_residual":
        err = (got.double().cpu() - ref).abs().max().item() / ref.abs().max().item()
        assert err <= 8e-3, err


# tile counts past one per CU (the persistent grid walks several tiles per workgroup; 297 is not a
# multiple of 8, so the XCD-contiguous order is off), every epilogue mode
@pytest.mark.parametrize("shape", [(8192, 2304, 768), (256 * 33, 2304, 128), (2048, 3072, 64)])
@pytest.mark.parametrize("mode", ["bias", "residual", "dropout_residual", "gelu_aux", "gelu_deriv", "gelu_bwd",
                                  "mul_aux", "gelu_noaux"])
def test_gemm_bf16_g4_persistent_matches_g8(shape, mode, g4_restore):
    """the persistent four-wave GEMM (next tile's first K-tiles in flight during this tile's
    epilogue) gives the same bits as one workgroup per tile and as gemm256_kernel"""
    M, N, Kd = shape
    A = _rand(M, Kd, dtype=torch.bfloat16, seed=81).to(DEV)
    B = _rand(N, Kd, dtype=torch.bfloat16, seed=82).to(DEV)
    bias = _rand(N, seed=83).to(DEV)
    res = _rand(M, N, dtype=torch.bfloat16, seed=84).to(DEV)
    outs = []
    for g4, persist in (("gelu", True), ("gelu", False), ("off", True)):
        K.set_g4_mode(g4)
        K.set_g4_persist(persist)
        aux = res.clone() if mode in ("gelu_bwd", "mul_aux") else torch.zeros(M, N, dtype=torch.bfloat16, device=DEV)
        kw = dict(bias=bias)
        if mode == "residual":
            kw.update(residual=res)
        elif mode == "dropout_residual":
            kw.update(residual=res, dropout_p=0.1, seed=K.Seed(79, device=DEV), salt=7)
        elif mode == "gelu_aux":
            kw.update(act=K.ACT_GELU, aux=aux)
        elif mode == "gelu_deriv":
            kw.update(act=K.ACT_GELU_D, aux=aux)
        elif mode == "gelu_bwd":
            kw = dict(act=K.ACT_GELU_BWD, aux=aux)
        elif mode == "mul_aux":
            kw = dict(act=K.ACT_MUL_AUX, aux=aux)
        else:
            kw.update(act=K.ACT_GELU)
        outs.append((K.gemm(A, B, **kw), aux))
    torch.cuda.synchronize()
    for o, x in outs[1:]:
        assert torch.equal(outs[0][0], o), (outs[0][0].float() - o.float()).abs().max().item()
        assert torch.equal(outs[0][1], x)


@pytest.mark.parametrize("mode", ["gelu_aux", "gelu_deriv", "residual", "dropout_residual"])
def test_gemm_bf16_g4_epilogues_match_g8(mode, g4_restore):
    """the four-wave kernel's fused epilogues of the encoder forward Linears (FFN1: bias + GELU with
    the pre-activation to aux; attention output / FFN2: bias [+ hashed dropout] + residual) are
    bit-identical to gemm256_kernel's on the same inputs"""
    M, N, Kd = 768, 1024, 768
    A = _rand(M, Kd, dtype=torch.bfloat16, seed=51).to(DEV)
    B = _rand(N, Kd, dtype=torch.bfloat16, seed=52).to(DEV)
    bias = _rand(N, seed=53).to(DEV)
    res = _rand(M, N, dtype=torch.bfloat16, seed=54).to(DEV)
    outs = {}
    for g4 in ("1", "0"):
        # (the GELU mode is opt-in in the step, see gemm_g4.hip)
        K.set_g4_mode("gelu" if g4 == "1" else "off")
        aux = torch.zeros(M, N, dtype=torch.bfloat16, device=DEV)
        if mode == "gelu_aux":
            out = K.gemm(A, B, bias=bias, act=K.ACT_GELU, aux=aux)
        elif mode == "gelu_deriv":  # EPI 5: GELU with its derivative to aux
            out = K.gemm(A, B, bias=bias, act=K.ACT_GELU_D, aux=aux)
        elif mode == "residual":
            out = K.gemm(A, B, bias=bias, residual=res)
        else:
            out = K.gemm(A, B, bias=bias, residual=res, dropout_p=0.1, seed=K.Seed(77, device=DEV), salt=5)
        outs[g4] = (out, aux)
    torch.cuda.synchronize()
    assert torch.equal(outs["1"][0], outs["0"][0])
    assert torch.equal(outs["1"][1], outs["0"][1])
    ref = A.double().cpu() @ B.double().cpu().T + bias.double().cpu()
    if mode == "residual":
        ref = ref + res.double().cpu()
    if mode == "gelu_deriv":
        t = ref.clone().requires_grad_(True)
        torch.nn.functional.gelu(t).backward(torch.ones_like(t))
        assert (outs["1"][1].double().cpu() - t.grad).abs().max().item() <= 1.2 * 2.0 ** -7
        ref = torch.nn.functional.gelu(ref)
    if mode != "dropout_residual":
        got = outs["1"][1] if mode == "gelu_aux" else outs["1"][0]
        err = (got.double().cpu() - ref).abs().max().item() / ref.abs().max().item()
        assert err <= 8e-3, err


# (M, N, K) reaching each kernel family: the 256x128 MFMA kernel (ragged), the split-operand x6f
# kernel (fp32) / 256x256 kernels (bf16), a split-K product (long K, small output)
@pytest.mark.parametrize("shape", [(300, 256, 128), (1024, 768, 768), (256, 192, 8192)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_gemm_gelu_deriv_pair(shape, dtype):
    """MMFD_ACT_GELU_D / MMFD_ACT_MUL_AUX (the training FFN's forward GELU saving gelu'(z), and the
    backward multiplying by it) against the pre-activation pair ACT_GELU / ACT_GELU_BWD: the forward
    output is bit-identical in both precisions; in fp32 the saved derivative is gelu_grad_f of the
    same fp32 z, so the backward product is bit-identical too (with caller-supplied split planes as
    well); in bf16 both backward forms are within 1 bf16 ulp-scale of the fp64 reference"""
    M, N, Kd = shape
    x = _rand(M, Kd, dtype=dtype, seed=M + 71).to(DEV)
    w = _rand(N, Kd, dtype=dtype, seed=N + 72, scale=0.1).to(DEV)
    b = _rand(N, seed=73).to(DEV)
    dy = _rand(M, Kd, dtype=dtype, seed=74).to(DEV)
    w2 = _rand(Kd, N, dtype=dtype, seed=75, scale=0.1).to(DEV)  # stored [K][N]: trans_b
    d = torch.empty(M, N, device=DEV, dtype=dtype)
    pre = torch.empty(M, N, device=DEV, dtype=dtype)
    y_d = K.gemm(x, w, bias=b, act=K.ACT_GELU_D, aux=d)
    y_g = K.gemm(x, w, bias=b, act=K.ACT_GELU, aux=pre)
    torch.cuda.synchronize()
    assert torch.equal(y_d, y_g), (y_d.float() - y_g.float()).abs().max().item()
    t = pre.double().cpu().requires_grad_(True)
    torch.nn.functional.gelu(t).backward(torch.ones_like(t))
    tol = 1e-6 if dtype == torch.float32 else 1.2 * 2.0 ** -7
    assert (d.double().cpu() - t.grad).abs().max().item() <= tol * 1.2
    # the backward's dY W2 (blocks.linear_dx layout: the weight MN-contiguous)
    g_mul = K.gemm(dy, w2, trans_b=True, act=K.ACT_MUL_AUX, aux=d)
    g_pre = K.gemm(dy, w2, trans_b=True, act=K.ACT_GELU_BWD, aux=pre)
    torch.cuda.synchronize()
    if dtype == torch.float32:
        assert torch.equal(g_mul, g_pre), (g_mul - g_pre).abs().max().item()
        if K.split_eligible(dy):
            g_pl = K.gemm(dy, w2, trans_b=True, act=K.ACT_MUL_AUX, aux=d, a_planes=K.split3(dy),
                          b_planes=K.split3(w2))
            torch.cuda.synchronize()
            assert torch.equal(g_pl, g_pre)
    ref = (dy.double().cpu() @ w2.double().cpu()) * t.grad
    scale = ref.abs().max().item()
    for g in (g_mul, g_pre):
        err = (g.double().cpu() - ref).abs().max().item() / scale
        assert err <= (1e-5 if dtype == torch.float32 else 1.6e-2), err


def test_gemm_mul_aux_needs_aux():
    with pytest.raises((RuntimeError, ValueError)):
        K.gemm(torch.randn(64, 64, device=DEV), torch.randn(64, 64, device=DEV), act=K.ACT_MUL_AUX)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_gemm_splitk_long_k(dtype):
    # dW of a BERT-like layer: K (tokens) long, small output -> split-K path
    Kd, M, N = 8192, 256, 384
    A = _rand(Kd, M, dtype=dtype, seed=3); B = _rand(Kd, N, dtype=dtype, seed=4)
    ref = A.double().T @ B.double()
    out = K.gemm(A.to(DEV), B.to(DEV), trans_a=True, trans_b=True, out_dtype=torch.float32)
    torch.cuda.synchronize()
    err = (out.double().cpu() - ref).abs().max().item()
    assert err <= 2e-3 * math.sqrt(Kd / 1024), err


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", [(8192, 256, 384), (300, 768, 512), (4096, 2304, 768), (130, 40, 24), (64, 40, 36)])
@pytest.mark.parametrize("beta", [0.0, 1.0])
def test_gemm_fused_rowsum(dtype, shape, beta):
    """dW = dY^T X with the bias gradient sum_tokens dY fused (split-K and direct, MFMA and
    simple/unaligned paths); beta=1 accumulates like a shared parameter's second use."""
    Kd, M, N = shape
    A = _rand(Kd, M, dtype=dtype, seed=31); B = _rand(Kd, N, dtype=dtype, seed=32)
    rs0 = _rand(M, seed=33)
    rs = rs0.clone().to(DEV)
    out = K.gemm(A.to(DEV), B.to(DEV), trans_a=True, trans_b=True, out_dtype=torch.float32, a_rowsum=rs,
                 a_rowsum_beta=beta)
    torch.cuda.synchronize()
    ref = A.double().T @ B.double()
    assert (out.double().cpu() - ref).abs().max().item() <= 2e-3 * max(1.0, math.sqrt(Kd / 1024))
    rref = A.double().sum(0) + beta * rs0.double()
    assert (rs.double().cpu() - rref).abs().max().item() <= 1e-4 * math.sqrt(Kd)


def test_gemm_fused_rowsum_nontransposed_bf16():
    """row sums of a K-contiguous A (layout 0) on the bf16 256x256 path"""
    M, N, Kd = 512, 256, 640
    A = _rand(M, Kd, dtype=torch.bfloat16, seed=34); B = _rand(N, Kd, dtype=torch.bfloat16, seed=35)
    rs = torch.empty(M, device=DEV)
    K.gemm(A.to(DEV), B.to(DEV), out_dtype=torch.float32, a_rowsum=rs)
    torch.cuda.synchronize()
    assert (rs.double().cpu() - A.double().sum(1)).abs().max().item() <= 1e-4


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_gemm_epilogues(dtype):
    M, N, Kd = 300, 256, 128
    x = _rand(M, Kd, dtype=dtype, seed=5); w = _rand(N, Kd, dtype=dtype, seed=6, scale=0.1)
    b = _rand(N, seed=7)
    res = _rand(M, N, dtype=dtype, seed=8)
    base = x.double() @ w.double().T + b.double()
    # gelu + aux
    aux = torch.empty(M, N, device=DEV, dtype=dtype)
    y = K.gemm(x.to(DEV), w.to(DEV), bias=b.to(DEV), act=K.ACT_GELU, aux=aux)
    torch.cuda.synchronize()
    _close(aux, base, dtype, 1.0)
    _close(y, torch.nn.functional.gelu(base), dtype, 1.0)
    # relu + residual
    y = K.gemm(x.to(DEV), w.to(DEV), bias=b.to(DEV), act=K.ACT_RELU, residual=res.to(DEV))
    _close(y, base.clamp_min(0) + res.double(), dtype, 1.0)
    # beta accumulate
    c0 = res.to(DEV).clone()
    K.gemm(x.to(DEV), w.to(DEV), out=c0, beta=1.0)
    _close(c0, x.double() @ w.double().T + res.double(), dtype, 1.0)
    # gelu backward
    pre = base.to(dtype)
    gy = K.gemm(x.to(DEV), w.to(DEV), act=K.ACT_GELU_BWD, aux=pre.to(DEV))
    t = pre.double().requires_grad_(True)
    torch.nn.functional.gelu(t).backward(torch.ones_like(t))
    _close(gy, (x.double() @ w.double().T) * t.grad, dtype, 1.0)


@pytest.mark.parametrize("layout", ["nt", "nn", "tn"])
@pytest.mark.parametrize("Kd", [64, 96, 768])
def test_gemm_bf16_persistent_many_items(layout, Kd):
    """The persistent 256x256 bf16 kernel walks several output tiles per workgroup as one K-tile
    stream (more tiles than CUs; ragged last row/column tiles; K of one, two and twelve K-tiles),
    with the bias + GELU + aux register epilogue. Reference: fp64 matmul on the GPU."""
    M, N = 8192 + 136, 2304 + 40
    g = torch.Generator(device=DEV).manual_seed(40)
    x = torch.randn(M, Kd, device=DEV, generator=g).bfloat16()
    w = torch.randn(N, Kd, device=DEV, generator=g).mul(0.1).bfloat16()
    b = torch.randn(N, device=DEV, generator=g)
    if layout == "nt":
        ref = x.double() @ w.double().T
        A, B, kw = x, w, {}
    elif layout == "nn":  # B stored [K][N]
        ref = x.double() @ w.double().T
        A, B, kw = x, w.T.contiguous(), {"trans_b": True}
    else:  # A stored [K][M], B stored [K][N]
        ref = x.double() @ w.double().T
        A, B, kw = x.T.contiguous(), w.T.contiguous(), {"trans_a": True, "trans_b": True}
    aux = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    y = K.gemm(A, B, bias=b, act=K.ACT_GELU, aux=aux, **kw)
    pre = ref + b.double()
    torch.cuda.synchronize()
    e_aux = (aux.double() - pre).abs().max().item()
    e_y = (y.double() - torch.nn.functional.gelu(pre)).abs().max().item()
    scale = pre.abs().max().item()
    assert e_aux <= 1e-2 * scale and e_y <= 1e-2 * scale, (e_aux, e_y, scale)
    # fp32 output with residual, no activation
    res = torch.randn(M, N, device=DEV, generator=g)
    y32 = K.gemm(A, B, residual=res, out_dtype=torch.float32, **kw)
    torch.cuda.synchronize()
    assert (y32.double() - (ref + res.double())).abs().max().item() <= 1e-4 * scale


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_gemm_dropout_mask(dtype):
    M, N, Kd = 256, 128, 64
    x = _rand(M, Kd, dtype=dtype, seed=9); w = _rand(N, Kd, dtype=dtype, seed=10)
    seed = K.Seed(1234)
    salt = K.salt_of("test.gemm.dropout")
    y = K.gemm(x.to(DEV), w.to(DEV), dropout_p=0.1, seed=seed, salt=salt, out_dtype=torch.float32)
    torch.cuda.synchronize()
    keep = torch.from_numpy(keep_mask(1234, salt, (M, N), 0.1))
    ref = (x.double() @ w.double().T) * keep / 0.9
    _close(y, ref, torch.float32 if dtype == torch.float32 else torch.bfloat16)
    frac = keep.float().mean().item()
    assert 0.88 < frac < 0.92


def test_dropout_hash_host_matches_numpy():
    from oracle.dropout_hash import dropout_hash
    for seed, salt, idx in [(0, 0, 0), (1234, K.salt_of("x"), 17), (2**40 + 5, 2**63 + 11, 2**35 + 3)]:
        assert K.dropout_hash(seed, salt, idx) == int(dropout_hash(seed, salt, np.array([idx], dtype=np.uint64))[0])


def test_colsum():
    for dtype in (torch.float32, torch.bfloat16):
        X = _rand(5000, 300, dtype=dtype, seed=11)
        got = K.colsum(X.to(DEV))
        torch.cuda.synchronize()
        ref = X.double().sum(0)
        assert (got.double().cpu() - ref).abs().max().item() < 1e-2


# ---------------------------------------------------------------------------------------------
# attention
# ---------------------------------------------------------------------------------------------
def _attn_ref(q, k, v, H, scale, key_bias=None, keep=None, p=0.0):
    B, Lq, HD = q.shape
    D = HD // H
    qh = q.double().view(B, Lq, H, D).transpose(1, 2)
    kh = k.double().view(B, -1, H, D).transpose(1, 2)
    vh = v.double().view(B, -1, H, D).transpose(1, 2)
    s = qh @ kh.transpose(-1, -2) * scale
    if key_bias is not None:
        s = s + key_bias.double()[:, None, None, :]
    pr = torch.softmax(s, -1)
    lse = torch.logsumexp(s, -1)
    pd = pr * keep / (1 - p) if keep is not None else pr
    o = (pd @ vh).transpose(1, 2).reshape(B, Lq, HD)
    return o, lse


ATTN_CASES = [(2, 4, 128, 128, 64), (2, 8, 197, 197, 32), (3, 2, 13, 29, 64), (2, 8, 128, 197, 32),
              (1, 12, 70, 70, 64), (2, 4, 21, 33, 8), (2, 2, 40, 40, 16), (1, 3, 65, 130, 48),
              (1, 2, 260, 300, 64), (2, 16, 256, 256, 64),  # L > 256: streaming backward kernels
              (1, 2, 512, 512, 64),  # bf16 forward keeps up to 512 keys resident
              (2, 4, 197, 197, 64), (1, 2, 208, 208, 64)]  # 13 query blocks: the last one split over two waves


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", ATTN_CASES)
@pytest.mark.parametrize("masked", [False, True])
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_attention_fwd_bwd(dtype, case, masked, p):
    B, H, Lq, Lk, D = case
    q = _rand(B, Lq, H * D, dtype=dtype, seed=20)
    kv = _rand(B, Lk, 2 * H * D, dtype=dtype, seed=21)  # fused K|V buffer -> strided views
    k, v = kv[..., : H * D], kv[..., H * D:]
    dout = _rand(B, Lq, H * D, dtype=dtype, seed=22)
    scale = D ** -0.5
    kb = None
    if masked:
        lens = torch.randint(1, Lk + 1, (B,), generator=torch.Generator().manual_seed(3))
        mask = (torch.arange(Lk)[None, :] < lens[:, None]).long()
        kb = K.mask_to_bias(mask.to(DEV))
        kb_cpu = kb.cpu()
    else:
        kb_cpu = None
    seed = K.Seed(77)
    salt = K.salt_of("test.attn")
    keep = None
    if p > 0:
        keep = torch.from_numpy(attn_keep_mask(77, salt, (B, H, Lq, Lk), p)).double()
    qd, kvd, dod = q.to(DEV), kv.to(DEV), dout.to(DEV)
    o, lse = K.attn_fwd(qd, kvd[..., : H * D], kvd[..., H * D:], H, key_bias=kb, dropout_p=p, seed=seed, salt=salt)
    dq, dk, dv = K.attn_bwd(qd, kvd[..., : H * D], kvd[..., H * D:], o, lse, dod, H, key_bias=kb, dropout_p=p,
                            seed=seed, salt=salt)
    torch.cuda.synchronize()
    # reference on the kernel's (rounded) inputs
    qr = q.double().requires_grad_(True)
    kr = k.double().requires_grad_(True)
    vr = v.double().requires_grad_(True)
    oref, lref = _attn_ref(qr, kr, vr, H, scale, kb_cpu, keep, p)
    oref.backward(dout.double())
    _close(o, oref, dtype)
    assert (lse.double().cpu() - lref).abs().max().item() < (1e-4 if dtype == torch.float32 else 2e-2)
    _close(dq, qr.grad, dtype)
    _close(dk, kr.grad, dtype)
    _close(dv, vr.grad, dtype)


@pytest.mark.parametrize("case", [(4, 12, 128, 128, 64, True, 0.1), (3, 12, 197, 197, 64, False, 0.0),
                                  (2, 8, 128, 197, 32, True, 0.1), (2, 3, 208, 200, 48, True, 0.0),
                                  (2, 2, 17, 45, 64, False, 0.1), (2, 4, 140, 140, 64, True, 0.1)])
def test_attention_fp32_split_operands_error_matches_fp32_mfma(case):
    """fp32 attention on split bf16 operands (include/mmfd.h mmfd_set_fp32_attn_mode: every product
    from the hi/mid/lo planes, six MFMA products accumulated in fp32) against a float64 reference:
    output, lse and all three gradients may not exceed the fp32-MFMA kernels' own error on the same
    inputs by more than 1.5x (+1e-7 of the tensor's scale). Covers the encoder shapes (BERT L = 128
    with mask + dropout, ViT L = 197: an odd 16-row remainder), cross attention at the head's D = 32,
    D = 48 and the 208-row resident maximum."""
    B, H, Lq, Lk, D, masked, p = case
    q = _rand(B, Lq, H * D, seed=30)
    kv = _rand(B, Lk, 2 * H * D, seed=31)
    k, v = kv[..., : H * D], kv[..., H * D:]
    dout = _rand(B, Lq, H * D, seed=32)
    kb = kb_cpu = None
    if masked:
        lens = torch.randint(1, Lk + 1, (B,), generator=torch.Generator().manual_seed(4))
        mask = (torch.arange(Lk)[None, :] < lens[:, None]).long()
        kb = K.mask_to_bias(mask.to(DEV))
        kb_cpu = kb.cpu()
    seed, salt = K.Seed(78), K.salt_of("test.attn.x6")
    keep = torch.from_numpy(attn_keep_mask(78, salt, (B, H, Lq, Lk), p)).double() if p > 0 else None
    qd, kvd, dod = q.to(DEV), kv.to(DEV), dout.to(DEV)
    outs = {}
    old = K.set_fp32_attn_mode("split")
    try:
        for mode in ("split", "native"):
            K.set_fp32_attn_mode(mode)
            o, lse = K.attn_fwd(qd, kvd[..., : H * D], kvd[..., H * D:], H, key_bias=kb, dropout_p=p, seed=seed,
                                salt=salt)
            g = K.attn_bwd(qd, kvd[..., : H * D], kvd[..., H * D:], o, lse, dod, H, key_bias=kb, dropout_p=p,
                           seed=seed, salt=salt)
            outs[mode] = (o, lse) + tuple(g)
        torch.cuda.synchronize()
    finally:
        K.set_fp32_attn_mode(old)
    qr, kr, vr = (t.double().requires_grad_(True) for t in (q, k, v))
    oref, lref = _attn_ref(qr, kr, vr, H, D ** -0.5, kb_cpu, keep, p)
    oref.backward(dout.double())
    refs = (oref.detach(), lref, qr.grad, kr.grad, vr.grad)
    for i, name in enumerate(("o", "lse", "dq", "dk", "dv")):
        sc = refs[i].abs().max().item()
        err = {m: (outs[m][i].double().cpu() - refs[i]).abs().max().item() / sc for m in outs}
        assert err["split"] <= 1.5 * err["native"] + 1e-7, (name, err)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("L", [96, 300])
def test_attention_batch_strided_rel_bias(dtype, L):
    """additive bias per batch row [B, H, L, L] (DeBERTa c2p + p2c) next to the key mask, against
    a float64 softmax reference; the shared [H, L, L] form (MPNet) is the rel_bias_sb = 0 case"""
    B, H, D = 2, 3, 64
    q = _rand(B, L, H * D, dtype=dtype, seed=60)
    k = _rand(B, L, H * D, dtype=dtype, seed=61)
    v = _rand(B, L, H * D, dtype=dtype, seed=62)
    rb = _rand(B, H, L, L, seed=63)
    mask = torch.ones(B, L, dtype=torch.long)
    mask[1, L // 3:] = 0
    kb = K.mask_to_bias(mask.to(DEV))
    scale = (3 * D) ** -0.5
    o, _ = K.attn_fwd(q.to(DEV), k.to(DEV), v.to(DEV), H, scale=scale, key_bias=kb, rel_bias=rb.to(DEV))
    torch.cuda.synchronize()
    qh = q.double().view(B, L, H, D).transpose(1, 2)
    kh = k.double().view(B, L, H, D).transpose(1, 2)
    vh = v.double().view(B, L, H, D).transpose(1, 2)
    s = qh @ kh.transpose(-1, -2) * scale + rb.double() + kb.double().cpu()[:, None, None, :]
    ref = (torch.softmax(s, -1) @ vh).transpose(1, 2).reshape(B, L, H * D)
    _close(o, ref, dtype)


def test_deberta_bias_kernels():
    """mmfd_deberta_rel_bias (tiled gather of c2p / p2c at host indices), mmfd_mask_rows and
    mmfd_attn_fill_masked_rows against their definitions"""
    B, H, L, S = 2, 3, 150, 64
    c2p = _rand(H, B * L, 2 * S, seed=70)
    p2c = _rand(H, B * L, 2 * S, seed=71)
    g = torch.Generator().manual_seed(72)
    ci = torch.randint(0, 2 * S, (L, L), generator=g, dtype=torch.int32)
    pi = torch.randint(0, 2 * S, (L, L), generator=g, dtype=torch.int32)
    out = K.deberta_rel_bias(c2p.to(DEV), p2c.to(DEV), ci.to(DEV), pi.to(DEV), B, L, 0.125)
    torch.cuda.synchronize()
    cb = c2p.view(H, B, L, 2 * S).permute(1, 0, 2, 3)  # [B,H,L,2S]
    pb = p2c.view(H, B, L, 2 * S).permute(1, 0, 2, 3)
    ref = torch.gather(cb, -1, ci.long().expand(B, H, L, L)) * 0.125 + \
        torch.gather(pb, -1, pi.long().expand(B, H, L, L)).transpose(-1, -2) * 0.125
    assert (out.cpu() - ref).abs().max().item() < 1e-6
    x = _rand(B * L, 40, seed=73).to(DEV)
    m = (torch.rand(B * L, generator=g) > 0.3).long()
    y = K.mask_rows(x.clone(), m.to(DEV))
    assert torch.equal(y.cpu(), x.cpu() * m[:, None])
    v = _rand(B, L, H * 32, seed=74)
    o = _rand(B, L, H * 32, seed=75)
    mk = torch.ones(B, L, dtype=torch.long)
    mk[1, 100:] = 0
    of = K.attn_fill_masked_rows(v.to(DEV), o.clone().to(DEV), H, mk.to(DEV)).cpu()
    assert torch.equal(of[0], o[0]) and torch.equal(of[1, :100], o[1, :100])
    assert (of[1, 100:] - v[1].mean(0)).abs().max().item() < 1e-5


# ---------------------------------------------------------------------------------------------
# LayerNorm / misc
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("width,eps,R", [(256, 1e-5, 1000), (768, 1e-12, 1000), (384, 1e-5, 1000), (520, 1e-5, 1001),
                                         (1024, 1e-12, 999), (768, 1e-12, 20011)])
def test_layernorm(dtype, width, eps, R):
    """row-per-wave (fp32, bf16 > 128 chunks), two-rows-per-wave (bf16 33-128 chunks: 520 = 65 chunks
    with a partial third, 768 = 96, 1024 = 128) and narrow forms; odd row counts (a half-wave row
    group alone at the end), and more rows than the backward's grid (the grid-stride loop with the
    next row prefetched)"""
    x = _rand(R, width, dtype=dtype, seed=30, scale=2.0) + 0.5
    g = _rand(width, seed=31) * 0.1 + 1.0
    b = _rand(width, seed=32) * 0.1
    dy = _rand(R, width, dtype=dtype, seed=33)
    add = _rand(R, width, dtype=dtype, seed=34)
    y, mean, rstd = K.layernorm_fwd(x.to(DEV), g.to(DEV), b.to(DEV), eps)
    dg = torch.empty(width, device=DEV); db = torch.empty(width, device=DEV)
    dx = K.layernorm_bwd(dy.to(DEV), x.to(DEV), g.to(DEV), mean, rstd, dx_add=add.to(DEV), dgamma=dg, dbeta=db)
    torch.cuda.synchronize()
    xr = x.double().requires_grad_(True)
    gr = g.double().requires_grad_(True)
    br = b.double().requires_grad_(True)
    yr = torch.nn.functional.layer_norm(xr, (width,), gr, br, eps)
    yr.backward(dy.double())
    _close(y, yr, dtype, 1.0)
    _close(dx, xr.grad + add.double(), dtype, 1.0)
    assert (dg.double().cpu() - gr.grad).abs().max().item() < 1e-3 * R ** 0.5
    assert (db.double().cpu() - br.grad).abs().max().item() < 1e-3 * R ** 0.5


@pytest.mark.parametrize("B,L,D,dt", [(1, 512, 256, torch.bfloat16), (3, 197, 200, torch.float32),
                                       (2, 7, 520, torch.bfloat16), (2, 9, 12, torch.float32)])
def test_seq_mean_shapes(B, L, D, dt):
    """vector kernel (D % 8 == 0: one-block-per-row-of-chunks, partial last block) and the scalar
    fallback (D = 12); output into a wider buffer (ldo > D) as the fusion head's concat does"""
    x = _rand(B, L, D, seed=41).to(dt)
    buf = torch.zeros(B, D + 8, device=DEV, dtype=dt)
    K.seq_mean_fwd(x.to(DEV), out=buf[:, :D])
    torch.cuda.synchronize()
    ref = x.double().mean(1)
    tol = 1e-5 if dt == torch.float32 else 1e-2
    assert (buf[:, :D].double().cpu() - ref).abs().max().item() < tol
    assert (buf[:, D:] == 0).all()


def test_seq_mean_xent():
    x = _rand(4, 13, 256, seed=40)
    m = K.seq_mean_fwd(x.to(DEV))
    dx = K.seq_mean_bwd(torch.ones(4, 256, device=DEV), 13)
    torch.cuda.synchronize()
    assert torch.allclose(m.cpu(), x.mean(1), atol=1e-6)
    assert torch.allclose(dx.cpu(), torch.full((4, 13, 256), 1 / 13), atol=1e-7)
    logits = [_rand(8, 3, seed=50 + i) for i in range(4)]
    labels = torch.randint(0, 3, (8, 4), generator=torch.Generator().manual_seed(0))
    loss, dl = K.xent_fwd_bwd([l.to(DEV) for l in logits], labels.to(DEV))
    torch.cuda.synchronize()
    lr = [l.double().requires_grad_(True) for l in logits]
    tot = sum(torch.nn.functional.cross_entropy(lr[i], labels[:, i]) for i in range(4))
    tot.backward()
    assert abs(loss[0].item() - tot.item()) < 1e-5
    for i in range(4):
        assert torch.allclose(dl[i].double().cpu(), lr[i].grad, atol=1e-6)


def test_xent_absent_paths_use_reference_label_columns():
    """train.py:163-167: path idx is trained on labels[:, idx] whatever other paths are None
    (the kernel used the position in the shortened list)."""
    from mmfd.train import path_losses
    logits = [_rand(6, 3, seed=70 + i) for i in range(2)]
    labels = torch.randint(0, 3, (6, 4), generator=torch.Generator().manual_seed(3))
    outs = ((None, logits[0].to(DEV).requires_grad_(True)), (None, logits[1].to(DEV).requires_grad_(True)))
    loss = path_losses(outs, labels.to(DEV))
    loss[0].backward()
    torch.cuda.synchronize()
    lr = [l.double().requires_grad_(True) for l in logits]
    l1 = torch.nn.functional.cross_entropy(lr[0], labels[:, 1])
    l3 = torch.nn.functional.cross_entropy(lr[1], labels[:, 3])
    (l1 + l3).backward()
    got = loss.detach().cpu().double()
    want = torch.tensor([(l1 + l3).item(), 0.0, l1.item(), 0.0, l3.item()], dtype=torch.float64)
    assert (got - want).abs().max().item() < 1e-5, (got, want)
    assert torch.allclose(outs[0][1].grad.double().cpu(), lr[0].grad, atol=1e-6)
    assert torch.allclose(outs[1][1].grad.double().cpu(), lr[1].grad, atol=1e-6)


def test_adamw_loads_torch_optimizer_state():
    """A torch.optim.AdamW state_dict (CPU 'step' tensors) loads into mmfd AdamW and the
    next step matches torch continuing from the same state."""
    from mmfd.optim import AdamW
    ps = [_rand(300, seed=80), _rand(7, 11, seed=81)]
    gs = [_rand(300, seed=82), _rand(7, 11, seed=83)]
    ref = [p.clone().requires_grad_(True) for p in ps]
    opt = torch.optim.AdamW(ref, lr=1e-3, weight_decay=0.01)
    for r, g in zip(ref, gs):
        r.grad = g.clone()
    opt.step()
    import copy
    sd = copy.deepcopy(opt.state_dict())  # as read back from a checkpoint file (no shared tensors)
    dev = [r.detach().clone().to(DEV).requires_grad_(True) for r in ref]
    mine = AdamW(dev, lr=1e-3, weight_decay=0.01)
    mine.load_state_dict(sd)
    assert mine.state[dev[0]]["step"].device.type == "cpu"  # torch leaves it where it was loaded
    for r, d, g in zip(ref, dev, gs):
        r.grad = 2 * g
        d.grad = (2 * g).to(DEV)
    opt.step()
    mine.step()
    torch.cuda.synchronize()
    for r, d in zip(ref, dev):
        assert (r.detach() - d.detach().cpu()).abs().max().item() < 1e-6
    assert mine.state[dev[0]]["step"].device == dev[0].device and float(mine.state[dev[0]]["step"]) == 2.0


def test_adamw_matches_torch():
    ps = [_rand(1000, seed=60), _rand(37, 5, seed=61)]
    gs = [_rand(1000, seed=62), _rand(37, 5, seed=63)]
    ref = [p.clone().requires_grad_(True) for p in ps]
    opt = torch.optim.AdamW(ref, lr=1e-3, weight_decay=0.01)
    from mmfd.optim import AdamW
    dev = [p.clone().to(DEV).requires_grad_(True) for p in ps]
    myopt = AdamW(dev, lr=1e-3, weight_decay=0.01)
    for it in range(3):
        for r, d, g in zip(ref, dev, gs):
            r.grad = g * (it + 1)
            d.grad = (g * (it + 1)).to(DEV)
        opt.step()
        myopt.step()
    torch.cuda.synchronize()
    for r, d in zip(ref, dev):
        assert (r.detach() - d.detach().cpu()).abs().max().item() < 1e-6


@pytest.mark.parametrize("layout", ["nt", "nn", "tn", "tt"])
@pytest.mark.parametrize("shape", [(512, 768, 768), (1000, 520, 200), (300, 264, 1056), (768, 256, 4096),
                                   (256, 2304, 65536)])
def test_gemm_fp32_split_operands_error_matches_fp32_mfma(layout, shape):
    """fp32 GEMMs on split bf16 operands (x = hi + mid + lo, six products accumulated small-first,
    include/mmfd.h mmfd_set_fp32_gemm_mode) against an fp64 product: the error may not exceed the
    fp32 MFMA's own on the same inputs by more than 1.5x (+1e-7 of the output scale); covers
    ragged M/N tiles, K not a multiple of 64 (K-contiguous operands only), split-K over the six
    segments (the tall K = 65536 weight-gradient shape) and every operand layout."""
    M, N, Kd = shape
    ta, tb = layout[0] == "t", layout[1] == "t"
    if not K.x6_ok(M, N, Kd, ta, tb):
        pytest.skip("MN-contiguous operands need whole 32-row K-steps on the split path (fp32 MFMA used)")
    g = torch.Generator().manual_seed(M + N + Kd)
    A = torch.randn((Kd, M) if ta else (M, Kd), generator=g).to(DEV)
    B = (torch.randn((Kd, N) if tb else (N, Kd), generator=g) * 0.05).to(DEV)
    ref = (A.double().T if ta else A.double()) @ (B.double() if tb else B.double().T)
    outs = {}
    old = K.set_fp32_gemm_mode("split")
    try:
        for mode in ("split", "native"):
            K.set_fp32_gemm_mode(mode)
            outs[mode] = K.gemm(A, B, trans_a=ta, trans_b=tb)
        torch.cuda.synchronize()
    finally:
        K.set_fp32_gemm_mode(old)
    scale = ref.abs().max().item()
    err = {m: (o.double() - ref).abs().max().item() / scale for m, o in outs.items()}
    assert err["split"] <= 1.5 * err["native"] + 1e-7, err
    assert err["split"] <= 1e-5 * math.sqrt(Kd / 768), err


@pytest.mark.parametrize("layout,shape", [
    ("nn", (65536, 2304, 768)),    # BERT QKV forward at bs = 256 (512 sequences x 128 tokens)
    ("nn", (100864, 3072, 768)),   # ViT FFN1 forward (512 images x 197 tokens)
    ("nn", (100864, 768, 3072)),   # ViT FFN2 forward
    ("nt", (65536, 768, 3072)),    # BERT FFN1 dX (dPre [tokens, 3072] x W1)
    ("nt", (100864, 3072, 768)),   # ViT FFN2 dX (dY [tokens, 768] x W2)
    ("tt", (3072, 768, 100864)),   # ViT FFN1 dW: K over every image token row (split-K)
    ("tt", (2304, 768, 65536)),    # BERT QKV dW
    ("tt", (768, 3072, 65536))])   # BERT FFN2 dW
def test_gemm_fp32_split_operands_bench_shapes(layout, shape):
    """The split-operand fp32 GEMM at the bs = 256 step's own launch shapes (the
    full grids' XCD tile order, the split-K cost model at K = 65,536 / 100,864): error against an
    fp64 product within 1.5x of the fp32 MFMA's own (+1e-7 of the output scale), as
    test_gemm_fp32_split_operands_error_matches_fp32_mfma. Operands are drawn on the device."""
    M, N, Kd = shape
    ta, tb = layout[0] == "t", layout[1] == "t"
    assert K.x6_ok(M, N, Kd, ta, tb)
    g = torch.Generator(DEV).manual_seed(M + N + Kd)
    A = torch.randn((Kd, M) if ta else (M, Kd), generator=g, device=DEV)
    B = torch.randn((Kd, N) if tb else (N, Kd), generator=g, device=DEV) * 0.05
    ref = (A.double().T if ta else A.double()) @ (B.double() if tb else B.double().T)
    outs = {}
    old = K.set_fp32_gemm_mode("split")
    try:
        for mode in ("split", "native"):
            K.set_fp32_gemm_mode(mode)
            outs[mode] = K.gemm(A, B, trans_a=ta, trans_b=tb)
        torch.cuda.synchronize()
    finally:
        K.set_fp32_gemm_mode(old)
    scale = ref.abs().max().item()
    err = {m: (o.double() - ref).abs().max().item() / scale for m, o in outs.items()}
    print(f"{layout} {shape}: split {err['split']:.3e} native {err['native']:.3e}")
    assert err["split"] <= 1.5 * err["native"] + 1e-7, err
    del A, B, ref, outs
    torch.cuda.empty_cache()


def test_gemm_fp32_split_operands_epilogues_rowsum():
    """the split path keeps the fp32 epilogues (bias, GELU + saved pre-activation, residual, dropout,
    beta) and the fused bias-gradient row sums of op(A), with and without split-K"""
    old = K.set_fp32_gemm_mode("split")
    try:
        M, N, Kd = 520, 768, 384
        x = _rand(M, Kd, seed=51).to(DEV); w = _rand(N, Kd, seed=52, scale=0.1).to(DEV)
        b = _rand(N, seed=53).to(DEV); res = _rand(M, N, seed=54).to(DEV)
        base = x.double() @ w.double().T + b.double()
        aux = torch.empty(M, N, device=DEV)
        y = K.gemm(x, w, bias=b, act=K.ACT_GELU, aux=aux)
        assert (aux.double() - base).abs().max().item() <= 2e-5
        assert (y.double() - torch.nn.functional.gelu(base)).abs().max().item() <= 2e-5
        y = K.gemm(x, w, bias=b, residual=res)
        assert (y.double() - base - res.double()).abs().max().item() <= 2e-5
        c0 = res.clone()
        K.gemm(x, w, out=c0, beta=1.0)
        assert (c0.double() - (x.double() @ w.double().T + res.double())).abs().max().item() <= 2e-5
        seed = K.Seed(11)
        yd = K.gemm(x, w, dropout_p=0.1, seed=seed, salt=K.salt_of("x6"))
        K.set_fp32_gemm_mode("native")
        yn = K.gemm(x, w, dropout_p=0.1, seed=seed, salt=K.salt_of("x6"))
        K.set_fp32_gemm_mode("split")
        assert torch.equal(yd == 0, yn == 0)  # same counter-hash mask
        for Mt, splits in ((2048, 0), (2048, 4)):  # weight gradient dW = dY^T X with its bias gradient
            dy = _rand(Mt, 256, seed=55).to(DEV); xx = _rand(Mt, 512, seed=56).to(DEV)
            rs = torch.full((256,), 0.5, device=DEV)
            dw = K.gemm(dy, xx, trans_a=True, trans_b=True, splits=splits, a_rowsum=rs, a_rowsum_beta=1.0)
            torch.cuda.synchronize()
            ref = dy.double().T @ xx.double()
            assert (dw.double() - ref).abs().max().item() <= 1e-5 * ref.abs().max().item()
            assert (rs.double() - (0.5 + dy.double().sum(0))).abs().max().item() <= 1e-4
    finally:
        K.set_fp32_gemm_mode(old)


@pytest.mark.parametrize("case", ["fast", "ragged", "splitk", "gelu_bwd"])
def test_gemm_out_planes_equal_split_of_output(case):
    """the epilogue's split planes (out_planes) are bit-identical to split3 of the fp32 output it
    writes, on the full-tile fast path, the per-element path (ragged tiles), the split-K reduce and
    with the GELU-backward epilogue; write_out=False leaves the fp32 output untouched"""
    old = K.set_fp32_gemm_mode("split")
    try:
        if case == "splitk":
            A = _rand(4096, 256, seed=61).to(DEV); B = _rand(4096, 512, seed=62).to(DEV)
            kw = dict(trans_a=True, trans_b=True, splits=4)
            M, N = 256, 512
        else:
            M, N, Kd = (1024, 768, 512) if case != "ragged" else (1000, 776, 200)
            A = _rand(M, Kd, seed=63).to(DEV); B = _rand(N, Kd, seed=64, scale=0.1).to(DEV)
            kw = dict(bias=_rand(N, seed=65).to(DEV))
            if case == "gelu_bwd":
                kw = dict(act=K.ACT_GELU_BWD, aux=_rand(M, N, seed=66).to(DEV))
        ref = K.gemm(A, B, **kw)
        pl = torch.empty((3, M, N), device=DEV, dtype=torch.bfloat16)
        out = torch.full((M, N), 7.0, device=DEV)
        K.gemm(A, B, out=out, out_planes=pl, write_out=False, **kw)
        both = torch.empty((3, M, N), device=DEV, dtype=torch.bfloat16)
        out2 = K.gemm(A, B, out_planes=both, **kw)
        torch.cuda.synchronize()
        assert torch.equal(out2, ref)
        assert torch.equal(pl.view(torch.int16), K.split3(ref).view(torch.int16))
        assert torch.equal(both.view(torch.int16), pl.view(torch.int16))
        assert bool((out == 7.0).all())
        recon = pl[0].double() + pl[1].double() + pl[2].double()
        assert (recon - ref.double()).abs().max().item() <= 2 ** -23 * ref.abs().max().item()
    finally:
        K.set_fp32_gemm_mode(old)


@pytest.mark.parametrize("L", [128, 197, 300])
def test_attention_bwd_dqkv_planes(L):
    """fp32 attention backward writing the split planes of the packed [dq | dk | dv] gradient: bit-
    identical to split3 of the fp32 gradient (v2 kernels write them from their stores, L = 300 takes
    the v1 kernels and a split pass); planes_only leaves the fp32 buffer untouched"""
    B, H, D = 3, 4, 64
    g = torch.Generator().manual_seed(L)
    qkv = torch.randn(B, L, 3 * H * D, generator=g).to(DEV)
    q, k, v = qkv[..., :H * D], qkv[..., H * D:2 * H * D], qkv[..., 2 * H * D:]
    o, lse = K.attn_fwd(q, k, v, H)
    do = torch.randn(B, L, H * D, generator=g).to(DEV)
    dqkv = torch.empty_like(qkv)
    K.attn_bwd(q, k, v, o, lse, do, H, dq=dqkv[..., :H * D], dk=dqkv[..., H * D:2 * H * D], dv=dqkv[..., 2 * H * D:])
    pl = torch.empty((3, B * L, 3 * H * D), device=DEV, dtype=torch.bfloat16)
    d2 = torch.empty_like(qkv)
    K.attn_bwd(q, k, v, o, lse, do, H, dq=d2[..., :H * D], dk=d2[..., H * D:2 * H * D], dv=d2[..., 2 * H * D:],
               dqkv_planes=pl)
    torch.cuda.synchronize()
    assert torch.equal(d2, dqkv)
    ref = K.split3(dqkv.view(B * L, -1))
    assert torch.equal(pl.view(torch.int16), ref.view(torch.int16))
    d3 = torch.full_like(qkv, 5.0)
    pl2 = torch.empty_like(pl)
    K.attn_bwd(q, k, v, o, lse, do, H, dq=d3[..., :H * D], dk=d3[..., H * D:2 * H * D], dv=d3[..., 2 * H * D:],
               dqkv_planes=pl2, planes_only=True)
    torch.cuda.synchronize()
    assert torch.equal(pl2.view(torch.int16), ref.view(torch.int16))
    if L <= 256:
        assert bool((d3 == 5.0).all())


def test_gemm_planes_only_operand_fails_loudly_off_the_split_path():
    """an output written only as planes (write_out=False) is marked; a later GEMM that would read
    its unwritten fp32 copy (here: fp32 MFMA mode) raises instead of computing on garbage"""
    old = K.set_fp32_gemm_mode("split")
    try:
        x = _rand(512, 256, seed=71).to(DEV); w = _rand(384, 256, seed=72).to(DEV)
        pl = torch.empty((3, 512, 384), device=DEV, dtype=torch.bfloat16)
        y = K.gemm(x, w, out_planes=pl, write_out=False)
        w2 = _rand(128, 384, seed=73).to(DEV)
        ok = K.gemm(y, w2, a_planes=pl)  # split path: reads the planes
        ref = (x.double() @ w.double().T) @ w2.double().T
        torch.cuda.synchronize()
        assert (ok.double() - ref).abs().max().item() <= 1e-4 * ref.abs().max().item()
        K.set_fp32_gemm_mode("native")
        with pytest.raises(RuntimeError, match="only as split planes"):
            K.gemm(y, w2, a_planes=pl)
    finally:
        K.set_fp32_gemm_mode(old)


@pytest.mark.parametrize("width", [64, 768])
def test_layernorm_fwd_planes_equal_split_of_output(width):
    """the fp32 LayerNorm forward writing its output's split planes in the same pass: y and the
    statistics equal the plain kernel's, the planes equal split3(y) bit for bit"""
    R = 1000
    x = _rand(R, width, seed=81).to(DEV)
    g = (1.0 + 0.1 * _rand(width, seed=82)).to(DEV); b = (0.1 * _rand(width, seed=83)).to(DEV)
    y0, m0, r0 = K.layernorm_fwd(x, g, b, 1e-12)
    pl = torch.empty((3, R, width), device=DEV, dtype=torch.bfloat16)
    y1, m1, r1 = K.layernorm_fwd(x, g, b, 1e-12, planes=pl)
    torch.cuda.synchronize()
    assert torch.equal(y0, y1) and torch.equal(m0, m1) and torch.equal(r0, r1)
    assert torch.equal(pl.view(torch.int16), K.split3(y1).view(torch.int16))


@pytest.mark.parametrize("drop", [False, True])
def test_layernorm_bwd_planes_equal_split_of_gemm_operand(drop):
    """the fp32 LayerNorm backward writing the split planes of the gradient the next GEMMs read
    (dx_drop with dropout, else dx): outputs equal the plain kernel's, planes == split3 bit for bit"""
    R, W = 1000, 768
    x = _rand(R, W, seed=91).to(DEV); dy = _rand(R, W, seed=92).to(DEV); add = _rand(R, W, seed=93).to(DEV)
    g = (1.0 + 0.1 * _rand(W, seed=94)).to(DEV); b = torch.zeros(W, device=DEV)
    _, mean, rstd = K.layernorm_fwd(x, g, b, 1e-12)
    seed = K.Seed(5)
    kw = dict(dropout_p=0.1, seed=seed, salt=K.salt_of("lnb")) if drop else {}
    outs = []
    for planes in (None, torch.empty((3, R, W), device=DEV, dtype=torch.bfloat16)):
        dd = torch.empty_like(dy) if drop else None
        dgm, dbt = torch.empty(W, device=DEV), torch.empty(W, device=DEV)
        dx = K.layernorm_bwd(dy, x, g, mean, rstd, dx_add=add, dgamma=dgm, dbeta=dbt, dx_drop=dd, planes=planes, **kw)
        outs.append((dx, dd, dgm, dbt, planes))
    torch.cuda.synchronize()
    (dx0, dd0, g0, b0, _), (dx1, dd1, g1, b1, pl) = outs
    assert torch.equal(dx0, dx1) and torch.equal(g0, g1) and torch.equal(b0, b1)
    src = dd1 if drop else dx1
    if drop:
        assert torch.equal(dd0, dd1)
    assert torch.equal(pl.view(torch.int16), K.split3(src).view(torch.int16))


@pytest.mark.parametrize("L", [128, 197, 300])
def test_attention_fwd_output_planes(L):
    """fp32 attention forward writing its output's split planes (v2 kernels from their stores, the
    L = 300 streaming path by a split pass): o unchanged, planes == split3(o) bit for bit"""
    B, H, D = 2, 4, 64
    g = torch.Generator().manual_seed(L + 7)
    qkv = torch.randn(B, L, 3 * H * D, generator=g).to(DEV)
    q, k, v = qkv[..., :H * D], qkv[..., H * D:2 * H * D], qkv[..., 2 * H * D:]
    o0, l0 = K.attn_fwd(q, k, v, H)
    pl = torch.empty((3, B * L, H * D), device=DEV, dtype=torch.bfloat16)
    o1, l1 = K.attn_fwd(q, k, v, H, o_planes=pl)
    torch.cuda.synchronize()
    assert torch.equal(o0, o1) and torch.equal(l0, l1)
    assert torch.equal(pl.view(torch.int16), K.split3(o1.view(B * L, -1)).view(torch.int16))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_gemm_single_tile_weight_gradient_many_splits(dtype):
    """the fusion head's weight-gradient shape (256 x 256 over 50,432 rows): one output tile, split-K
    up to one round of blocks (more than the former cap of 32 splits), with the fused bias gradient
    accumulating onto a shared parameter's first use"""
    from mmfd.kernels import GemmArgs, dtype_code, lib
    import ctypes
    Kd, M, N = 50432, 256, 256
    dy = _rand(Kd, M, dtype=dtype, seed=71).to(DEV); xx = _rand(Kd, N, dtype=dtype, seed=72).to(DEV)
    a = GemmArgs()
    a.dtype, a.c_dtype = dtype_code(dtype), dtype_code(torch.float32)
    a.trans_a, a.trans_b = 1, 1
    a.M, a.N, a.K = M, N, Kd
    a.A, a.lda, a.B, a.ldb = dy.data_ptr(), M, xx.data_ptr(), N
    assert lib().mmfd_gemm_splits(ctypes.byref(a)) > 32
    rs = torch.full((M,), 0.25, device=DEV)
    dw = K.gemm(dy, xx, trans_a=True, trans_b=True, out_dtype=torch.float32, a_rowsum=rs, a_rowsum_beta=1.0)
    torch.cuda.synchronize()
    ref = dy.double().T @ xx.double()
    tol = (1e-5 if dtype == torch.float32 else 2e-3) * ref.abs().max().item()
    assert (dw.double() - ref).abs().max().item() <= tol
    assert (rs.double() - (0.25 + dy.double().sum(0))).abs().max().item() <= 1e-4 * math.sqrt(Kd)


def _pack_keep_bits(keep, Lk):
    """oracle keep mask [B, H, Lq, Lk] (bool) -> the drop_mask words [B*H*Lq, ceil(Lk/32)] (uint32)"""
    import numpy as np
    W = (Lk + 31) // 32
    k = np.zeros(keep.shape[:-1] + (W * 32,), dtype=np.uint64)
    k[..., :Lk] = keep
    k = k.reshape(-1, W, 32)
    return (k << np.arange(32, dtype=np.uint64)).sum(axis=2).astype(np.uint32)


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("B,H,L,D", [(4, 12, 128, 64), (3, 8, 197, 32), (2, 4, 300, 64)])
def test_attention_dropout_keep_bitmask(dtype, B, H, L, D):
    """the forward writes the dropout keep-mask once as a bitmask
    (mmfd_attn_args.drop_mask) and the backward reads it instead of re-hashing. The words equal the
    oracle's counter-hash mask (oracle/dropout_hash.attn_keep_mask: one hash per key pair) bit for bit on every valid key, and
    output, lse, dQ, dK and dV are bit-identical with and without the mask — BERT's shape (the
    split-operand / bf16 resident kernels, mask staged in LDS by dK/dV), the head's D = 32 at
    L = 197 (fp32: dK/dV has no LDS left for the mask and re-hashes), and L = 300 (the streaming
    kernels, whose forward does not hash into the mask: a fill pass writes it)."""
    import numpy as np
    dt = torch.float32 if dtype == "fp32" else torch.bfloat16
    g = torch.Generator(DEV).manual_seed(B * 1000 + L)
    q = torch.randn(B, L, H * D, generator=g, device=DEV).to(dt)
    kv = torch.randn(B, L, 2 * H * D, generator=g, device=DEV).to(dt)
    do = torch.randn(B, L, H * D, generator=g, device=DEV).to(dt)
    lens = torch.randint(L // 2, L + 1, (B,), generator=torch.Generator().manual_seed(L))
    kb = torch.where(torch.arange(L)[None] < lens[:, None], 0.0, -10000.0).to(DEV)
    p, seed, salt = 0.1, K.Seed(91), K.salt_of("test.attn.bitmask")
    k, v = kv[..., :H * D], kv[..., H * D:]
    res = {}
    for use in (False, True):
        dm = K.drop_mask_buffer(B, H, L, L, DEV) if use else None
        o, lse = K.attn_fwd(q, k, v, H, key_bias=kb, dropout_p=p, seed=seed, salt=salt, drop_mask=dm)
        dq, dk, dv = K.attn_bwd(q, k, v, o, lse, do, H, key_bias=kb, dropout_p=p, seed=seed, salt=salt, drop_mask=dm)
        torch.cuda.synchronize()
        res[use] = (o, lse, dq, dk, dv, dm)
    for a, b in zip(res[False][:5], res[True][:5]):
        assert torch.equal(a, b), (a.float() - b.float()).abs().max().item()
    words = res[True][5].cpu().numpy().view(np.uint32).reshape(B, H * L, -1)
    want = _pack_keep_bits(attn_keep_mask(91, salt, (B, H, L, L), p), L).reshape(B, H * L, -1)
    # compared on the keys a query attends to (the bf16 resident forward records the mask from P,
    # whose masked-out keys are 0 whatever the hash: their backward P is 0 as well)
    for b in range(B):
        valid = _pack_keep_bits(np.arange(L)[None, None, None, :] < int(lens[b]), L).reshape(-1)
        assert np.array_equal(words[b] & valid, want[b] & valid), b


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,L,D,V", [(8, 64, 768, 50), (3, 37, 100, 50), (1, 1, 64, 50), (16, 128, 200, 3),
                                     (4, 100, 768, 2), (40, 128, 64, 2), (40, 128, 64, 1)])
def test_embed_bwd_deterministic_scatter_add(dtype, B, L, D, V):
    """csrc/embed_bwd.hip: the embedding tables' gradients (word: sort rows by id, one writer per id;
    type: ordered slab partials; position: batch order) equal an fp64 index_add of the same rows, add
    into what the tables held, skip padding rows, and repeat bit for bit (heavily repeated ids; V = 2-3:
    runs of hundreds of rows across many 32-row pieces, the padding id's run included)."""
    g = torch.Generator().manual_seed(B * 1000 + L)
    ids = torch.randint(0, V, (B, L), generator=g).cuda()
    tts = torch.randint(0, 2, (B, L), generator=g).cuda()
    dsum = (torch.randn(B, L, D, generator=g)).to(dtype).cuda()
    base = [torch.randn(V, D, generator=g).cuda(), torch.randn(L, D, generator=g).cuda(),
            torch.randn(2, D, generator=g).cuda()]
    outs = []
    for _ in range(2):
        dword, dpos, dtyp = (t.clone() for t in base)
        K.embed_bwd(ids, tts, dsum, dword, dpos, dtyp, padding_idx=0)
        torch.cuda.synchronize()
        outs.append((dword, dpos, dtyp))
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    x = dsum.double().reshape(B * L, D).cpu()
    i = ids.reshape(-1).cpu()
    keep = i != 0
    rw = base[0].double().cpu().index_add(0, i[keep], x[keep])
    rp = base[1].double().cpu() + x.reshape(B, L, D).sum(0)
    rt = base[2].double().cpu().index_add(0, tts.reshape(-1).cpu(), x)
    for got, ref in zip(outs[0], (rw, rp, rt)):
        err = (got.double().cpu() - ref).abs().max().item()
        assert err <= 1e-5 * max(1.0, ref.abs().max().item()), err
    # NULL tables are skipped
    dword = base[0].clone()
    K.embed_bwd(ids, None, dsum, dword, None, None, padding_idx=-1)
    torch.cuda.synchronize()
    rw = base[0].double().cpu().index_add(0, i, x)
    assert (dword.double().cpu() - rw).abs().max().item() <= 1e-5 * max(1.0, rw.abs().max().item())


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_gemm_ext_acts_full_epilogue_through_reduce(dtype):
    """MMFD_ACT_MUL_AUX / MMFD_ACT_GELU_D off the four-wave kernel run through a split-K slab and the
    reduce's epilogue (gemm.hip epilogue_store8_x): with dropout, a residual and beta the result equals
    the tile kernels' GELU_BWD / GELU path on the same inputs — bit for bit in fp32 (the saved
    derivative is gelu_grad_f of the same fp32 pre-activation), within bf16 rounding in bf16"""
    M, N, Kd = 512, 384, 256  # N not a multiple of 256: never the four-wave kernel
    x = _rand(M, Kd, dtype=dtype, seed=91).to(DEV)
    w = _rand(N, Kd, dtype=dtype, seed=92, scale=0.1).to(DEV)
    b = _rand(N, seed=93).to(DEV)
    res = _rand(M, N, dtype=dtype, seed=94).to(DEV)
    pre = torch.empty(M, N, device=DEV, dtype=dtype)
    d = torch.empty(M, N, device=DEV, dtype=dtype)
    seed = K.Seed(95, device=DEV)
    kw = dict(bias=b, residual=res, dropout_p=0.1, seed=seed, salt=9)
    y_g = K.gemm(x, w, act=K.ACT_GELU, aux=pre, **kw)
    y_d = K.gemm(x, w, act=K.ACT_GELU_D, aux=d, **kw)
    torch.cuda.synchronize()
    if dtype == torch.float32:
        assert torch.equal(y_g, y_d), (y_g - y_d).abs().max().item()
    else:
        assert (y_g.float() - y_d.float()).abs().max().item() <= y_g.float().abs().max().item() * 2.0 ** -7
    dy = _rand(M, Kd, dtype=dtype, seed=96).to(DEV)
    w2 = _rand(Kd, N, dtype=dtype, seed=97, scale=0.1).to(DEV)
    c0 = _rand(M, N, dtype=dtype, seed=98).to(DEV)
    c1, c2 = c0.clone(), c0.clone()
    K.gemm(dy, w2, trans_b=True, act=K.ACT_GELU_BWD, aux=pre, out=c1, beta=1.0, **kw)
    K.gemm(dy, w2, trans_b=True, act=K.ACT_MUL_AUX, aux=d, out=c2, beta=1.0, **kw)
    torch.cuda.synchronize()
    if dtype == torch.float32:
        assert torch.equal(c1, c2), (c1 - c2).abs().max().item()
    else:
        assert (c1.float() - c2.float()).abs().max().item() <= c1.float().abs().max().item() * 2.0 ** -6
