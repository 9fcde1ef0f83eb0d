"""Implicit-GEMM convolution (mmfd_gemm_args.conv, csrc/gemm_tiles.h ConvFill / XfConvFill) — the
ResNet50 extractor's 3x3 and strided 1x1 convolutions (im2im_retrieval.py:14-17, 29-36) without the
im2col matrix.

Parity: the window-gathering fill stages exactly the values im2col_nhwc would have written, in the
same K order, into the same kernels' LDS images — so against the explicit im2col + GEMM on the same
kernel family the result is BIT-IDENTICAL (fp32 on the fp32-MFMA 256x128 kernel and on the
split-operand x6f kernel; bf16 on the 256x128 kernel). bf16 products that the explicit path runs on
the 256x256 kernels are checked at 1 bf16 ulp of the output scale. Against torch's fp64 conv2d
(F.conv2d on the CPU, the reference's arithmetic in higher precision): fp32 within 1e-5 of the output
scale, bf16 within 8e-3.
"""
import pytest
import torch
import torch.nn.functional as F

from mmfd import kernels as K

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _case(N, H, W, C, Cout, k, stride, pad, dtype, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(N, H, W, C, generator=g)
    w = torch.randn(Cout, C, k, k, generator=g) / (k * k * C) ** 0.5
    b = torch.randn(Cout, generator=g)
    wg = w.permute(0, 2, 3, 1).reshape(Cout, k * k * C)  # (kh, kw, c) columns, as conv_weight_prep
    return x, w, b, wg


# (N, H, W, C, Cout, k, stride, pad): the ResNet50 shapes that take each kernel, small batches;
# rows N*Ho*Wo deliberately not a multiple of the 256-row tile
SHAPES = [
    (3, 56, 56, 64, 64, 3, 1, 1),      # layer1 conv2 (256x128 kernel)
    (2, 56, 56, 128, 128, 3, 2, 1),    # layer2 first conv2, stride 2
    (5, 14, 14, 256, 256, 3, 1, 1),    # layer3 conv2 (fp32: split-operand x6f)
    (3, 7, 7, 512, 512, 3, 1, 1),      # layer4 conv2, padding on every border row
    (4, 28, 28, 256, 512, 1, 2, 0),    # layer3 downsample 1x1 stride 2
    (2, 13, 11, 96, 320, 3, 2, 1),     # odd sizes: H != W, ragged windows
]


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", SHAPES)
def test_conv_implicit_equals_im2col_gemm(shape, dtype):
    N, H, W, C, Cout, k, stride, pad = shape
    if not K.conv_implicit_ok(dtype, C):
        pytest.skip("channel count not eligible for this dtype")
    x, w, b, wg = _case(N, H, W, C, Cout, k, stride, pad, dtype, seed=N * 1000 + C + Cout)
    xd = x.reshape(-1, C).to(DEV, dtype).contiguous()
    wd = wg.to(DEV, dtype).contiguous()
    bd = b.to(DEV)
    y, Ho, Wo = K.conv2d_nhwc(xd, N, H, W, C, wd, k, stride, pad, bias=bd, act=K.ACT_RELU)
    cols, Ho2, Wo2 = K.im2col_nhwc(xd, N, H, W, C, k, stride, pad)
    ref_gemm = K.gemm(cols, wd, bias=bd, act=K.ACT_RELU)
    torch.cuda.synchronize()
    assert (Ho, Wo) == (Ho2, Wo2)
    M = N * Ho * Wo
    same_family = dtype == torch.float32 or (Cout <= 128 and M >= 4096)  # gemm.hip use_g8
    if same_family:
        assert torch.equal(y, ref_gemm), (y.float() - ref_gemm.float()).abs().max().item()
    else:
        ulp = ref_gemm.float().abs().max().item() * 2.0 ** -7
        assert (y.float() - ref_gemm.float()).abs().max().item() <= ulp
    # against fp64 conv2d on the CPU (the same bf16-rounded operands for the bf16 case)
    xr = xd.double().cpu().reshape(N, H, W, C).permute(0, 3, 1, 2)
    wr = wd.double().cpu().reshape(Cout, k, k, C).permute(0, 3, 1, 2)
    ref = F.relu(F.conv2d(xr, wr, b.double(), stride=stride, padding=pad)).permute(0, 2, 3, 1).reshape(M, Cout)
    err = (y.double().cpu() - ref).abs().max().item() / ref.abs().max().item()
    assert err <= (1e-5 if dtype == torch.float32 else 8e-3), err


def test_conv_implicit_residual_first_and_planes():
    """the bottleneck epilogue relu(conv + bias + identity) (residual_first) and caller-supplied
    activation planes (split3(x)) on the split-operand path give the same bits as the plain call"""
    N, H, W, C, Cout, k = 4, 14, 14, 256, 256, 3
    x, w, b, wg = _case(N, H, W, C, Cout, k, 1, 1, torch.float32, seed=7)
    xd, wd, bd = x.reshape(-1, C).to(DEV), wg.to(DEV).contiguous(), b.to(DEV)
    ident = torch.randn(N * H * W, Cout, generator=torch.Generator().manual_seed(8)).to(DEV)
    y1, _, _ = K.conv2d_nhwc(xd, N, H, W, C, wd, k, 1, 1, bias=bd, act=K.ACT_RELU, residual=ident,
                             residual_first=True)
    y2, _, _ = K.conv2d_nhwc(xd, N, H, W, C, wd, k, 1, 1, bias=bd, act=K.ACT_RELU, residual=ident,
                             residual_first=True, x_planes=K.split3(xd))
    cols, _, _ = K.im2col_nhwc(xd, N, H, W, C, k, 1, 1)
    y3 = K.gemm(cols, wd, bias=bd, act=K.ACT_RELU, residual=ident, residual_first=True)
    torch.cuda.synchronize()
    assert torch.equal(y1, y2) and torch.equal(y1, y3)


def test_conv_implicit_rejects_bad_geometry():
    """a channel count that would let a K-step straddle two filter taps, or a weight of the wrong
    width, is refused instead of computed"""
    xd = torch.randn(2 * 8 * 8, 48, device=DEV)
    with pytest.raises(ValueError):
        K.conv2d_nhwc(xd, 2, 8, 8, 48, torch.randn(64, 9 * 48, device=DEV), 3, 1, 1)
    xd = torch.randn(2 * 8 * 8, 64, device=DEV)
    with pytest.raises(ValueError):
        K.conv2d_nhwc(xd, 2, 8, 8, 64, torch.randn(64, 9 * 64 + 8, device=DEV), 3, 1, 1)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("N", [64, 48, 16])
@pytest.mark.parametrize("trans_a", [False, True])
def test_gemm_narrow_tile(N, trans_a, dtype):
    """tall GEMMs with N <= 64 and K-contiguous B run on the 256x64 tile (gemm_mfma_n64_kernel: the
    ResNet stem and layer-1 convolutions, 1x1 and 3x3): against fp64, ragged M and K, with the
    bias + ReLU epilogue and split-K"""
    M, Kd = 4096 + 200, 152
    g = torch.Generator().manual_seed(N + 3 * int(trans_a))
    A = torch.randn((Kd, M) if trans_a else (M, Kd), generator=g)
    B = torch.randn(N, Kd, generator=g) / Kd ** 0.5
    b = torch.randn(N, generator=g)
    Ad, Bd = A.to(DEV, dtype), B.to(DEV, dtype)
    ref = F.relu((Ad.double().cpu().T if trans_a else Ad.double().cpu()) @ Bd.double().cpu().T + b.double())
    for splits in (0, 3):
        y = K.gemm(Ad, Bd, trans_a=trans_a, bias=b.to(DEV), act=K.ACT_RELU, splits=splits)
        torch.cuda.synchronize()
        err = (y.double().cpu() - ref).abs().max().item() / ref.abs().max().item()
        assert err <= (1e-5 if dtype == torch.float32 else 8e-3), (splits, err)
