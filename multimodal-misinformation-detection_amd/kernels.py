"""Host bindings of libmmfd_hip.so (the C ABI declared in include/mmfd.h) plus thin torch-tensor
wrappers. PyTorch only provides device memory, the current HIP stream and autograd plumbing; every
computation below is a launch of one of our gfx950 kernels.

Two layers over the same C ABI:
  * the training / retrieval hot path (GEMM, attention, LayerNorm, cross entropy, AdamW, sequence
    mean, cast, cosine scores, top-k) goes through the PyTorch custom ops torch.ops.mmfd.* that
    libmmfd_torch.so registers (csrc/torch_ops.cpp: TORCH_LIBRARY schemas with declared
    mutations, CUDA/HIP dispatch; fake kernels in mmfd/ops.py);
  * the remaining entry points (encoder embeddings, ResNet / Swinv2 / DeBERTa helpers,
    preprocessing) are called through ctypes.

There is no fallback: if either shared library is missing or cannot be loaded, every op raises
`NativeLibraryError` (the product path must never silently run on something else).
"""
from __future__ import annotations

import ctypes
import os
import zlib

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MMFD_LIB_PATH") or os.path.join(_HERE, "libmmfd_hip.so")  # env override: A/B runs of two builds (tools/ab.sh)
TORCH_LIB_PATH = os.path.join(os.path.dirname(LIB_PATH), "libmmfd_torch.so")

F32, BF16, F16 = 0, 1, 2
ABI_VERSION = 3  # include/mmfd.h MMFD_ABI_VERSION: the layout of the argument structs below
COS_PAIR, COS_NORMALIZED, COS_ROUND_F16 = 0, 1, 4
ACT_NONE, ACT_GELU, ACT_RELU, ACT_GELU_BWD, ACT_RELU_BWD, ACT_TANH, ACT_SIGMOID = 0, 1, 2, 3, 4, 5, 6
# GELU whose aux keeps gelu'(pre-activation), and its backward (out *= aux): the training FFNs
ACT_GELU_D, ACT_MUL_AUX = 7, 8


class NativeLibraryError(RuntimeError):
    pass


class EpilogueArgs(ctypes.Structure):
    _fields_ = [
        ("bias", ctypes.c_void_p),
        ("residual", ctypes.c_void_p), ("ldr", ctypes.c_int64),
        ("aux", ctypes.c_void_p), ("ldaux", ctypes.c_int64),
        ("act", ctypes.c_int),
        ("dropout_p", ctypes.c_float),
        ("seed", ctypes.c_void_p),
        ("salt", ctypes.c_uint64),
        ("residual_first", ctypes.c_int),
        ("out_planes", ctypes.c_void_p),
    ]


class _Sized(ctypes.Structure):
    """argument structs that start with `struct_size` (include/mmfd.h, ABI version 2): set on
    construction, so the library can refuse a caller built against another layout"""

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        if "struct_size" not in kw:
            self.struct_size = ctypes.sizeof(self)


class GemmArgs(_Sized):
    _fields_ = [
        ("struct_size", ctypes.c_int64),
        ("dtype", ctypes.c_int), ("trans_a", ctypes.c_int), ("trans_b", ctypes.c_int),
        ("M", ctypes.c_int64), ("N", ctypes.c_int64), ("K", ctypes.c_int64),
        ("A", ctypes.c_void_p), ("lda", ctypes.c_int64),
        ("B", ctypes.c_void_p), ("ldb", ctypes.c_int64),
        ("C", ctypes.c_void_p), ("ldc", ctypes.c_int64), ("c_dtype", ctypes.c_int),
        ("alpha", ctypes.c_float), ("beta", ctypes.c_float),
        ("ep", EpilogueArgs),
        ("workspace", ctypes.c_void_p), ("workspace_bytes", ctypes.c_int64),
        ("splits", ctypes.c_int),
        ("a_rowsum", ctypes.c_void_p), ("a_rowsum_beta", ctypes.c_float),
        ("a_planes", ctypes.c_void_p), ("b_planes", ctypes.c_void_p),
        ("a_planes_only", ctypes.c_int), ("b_planes_only", ctypes.c_int),
        ("conv", ctypes.c_void_p),  # const mmfd_conv_geom* (ABI 3): implicit-GEMM convolution
    ]


class ConvGeomArgs(ctypes.Structure):
    """include/mmfd.h mmfd_conv_geom"""
    _fields_ = [("N", ctypes.c_int64), ("H", ctypes.c_int64), ("W", ctypes.c_int64), ("C", ctypes.c_int64),
                ("KH", ctypes.c_int), ("KW", ctypes.c_int), ("stride", ctypes.c_int), ("pad", ctypes.c_int),
                ("Ho", ctypes.c_int64), ("Wo", ctypes.c_int64)]


class AttnArgs(_Sized):
    _fields_ = [
        ("struct_size", ctypes.c_int64),
        ("dtype", ctypes.c_int),
        ("B", ctypes.c_int64), ("H", ctypes.c_int64), ("Lq", ctypes.c_int64), ("Lk", ctypes.c_int64),
        ("D", ctypes.c_int64),
        ("scale", ctypes.c_float),
        ("q", ctypes.c_void_p), ("q_sb", ctypes.c_int64), ("q_st", ctypes.c_int64),
        ("k", ctypes.c_void_p), ("k_sb", ctypes.c_int64), ("k_st", ctypes.c_int64),
        ("v", ctypes.c_void_p), ("v_sb", ctypes.c_int64), ("v_st", ctypes.c_int64),
        ("o", ctypes.c_void_p), ("o_sb", ctypes.c_int64), ("o_st", ctypes.c_int64),
        ("lse", ctypes.c_void_p),
        ("key_bias", ctypes.c_void_p),
        ("rel_bias", ctypes.c_void_p),
        ("dropout_p", ctypes.c_float), ("seed", ctypes.c_void_p), ("salt", ctypes.c_uint64),
        ("dout", ctypes.c_void_p), ("do_sb", ctypes.c_int64), ("do_st", ctypes.c_int64),
        ("dq", ctypes.c_void_p), ("dq_sb", ctypes.c_int64), ("dq_st", ctypes.c_int64),
        ("dk", ctypes.c_void_p), ("dk_sb", ctypes.c_int64), ("dk_st", ctypes.c_int64),
        ("dv", ctypes.c_void_p), ("dv_sb", ctypes.c_int64), ("dv_st", ctypes.c_int64),
        ("delta", ctypes.c_void_p),
        ("d_rel_bias", ctypes.c_void_p),
        ("accumulate_dq", ctypes.c_int),
        ("accumulate_dkv", ctypes.c_int),
        ("rel_bias_sb", ctypes.c_int64),
        ("rel_bias_mod", ctypes.c_int64),
        ("cos_logit_scale", ctypes.c_void_p),
        ("cos_max_log", ctypes.c_float),
        ("dqkv_planes", ctypes.c_void_p), ("planes_only", ctypes.c_int),
        ("o_planes", ctypes.c_void_p),
        ("drop_mask", ctypes.c_void_p),
    ]


class AdamWTensor(ctypes.Structure):
    _fields_ = [
        ("param", ctypes.c_void_p), ("grad", ctypes.c_void_p), ("exp_avg", ctypes.c_void_p),
        ("exp_avg_sq", ctypes.c_void_p), ("param_bf16", ctypes.c_void_p), ("step", ctypes.c_void_p),
        ("numel", ctypes.c_int64),
    ]


_VP, _I64, _I, _F, _U64 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_float, ctypes.c_uint64

# name -> (restype, argtypes); every symbol declared in include/mmfd.h
SIGNATURES = {
    "mmfd_last_error_string": (ctypes.c_char_p, []),
    "mmfd_version": (_I, []),
    "mmfd_dropout_hash": (ctypes.c_uint32, [_U64, _U64, _U64]),
    "mmfd_gemm": (_I, [ctypes.POINTER(GemmArgs), _VP]),
    "mmfd_gemm_workspace_bytes": (_I64, [ctypes.POINTER(GemmArgs)]),
    "mmfd_set_fp32_gemm_mode": (_I, [_I]),
    "mmfd_set_fp32_attn_mode": (_I, [_I]),
    "mmfd_gemm_splits": (_I, [ctypes.POINTER(GemmArgs)]),
    "mmfd_gemm_runs_split": (_I, [ctypes.POINTER(GemmArgs)]),
    "mmfd_set_g4_mode": (_I, [_I]),
    "mmfd_set_g4_persist": (_I, [_I]),
    "mmfd_transpose": (_I, [_I, _I64, _I64, _VP, _I64, _VP, _I64, _VP]),
    "mmfd_set_g4_kmax": (_I64, [_I64]),
    "mmfd_split3": (_I, [_I64, _I64, _VP, _I64, _VP, _VP]),
    "mmfd_layernorm_fwd_split": (_I, [_I64, _I64, _VP, _I64, _VP, _VP, _F, _VP, _I64, _VP, _VP, _VP, _VP]),
    "mmfd_layernorm_bwd_split": (_I, [_I64, _I64, _VP, _I64, _VP, _I64, _VP, _VP, _VP, _VP, _I64, _VP, _I64, _VP, _VP,
                                      _F, _VP, _F, _VP, _U64, _VP, _I64, _VP, _VP]),
    "mmfd_colsum": (_I, [_I, _I64, _I64, _VP, _I64, _VP, _F, _VP, _I64, _VP]),
    "mmfd_attn_fwd": (_I, [ctypes.POINTER(AttnArgs), _VP]),
    "mmfd_attn_bwd": (_I, [ctypes.POINTER(AttnArgs), _VP]),
    "mmfd_layernorm_fwd": (_I, [_I, _I64, _I64, _VP, _I64, _VP, _VP, _F, _VP, _I64, _VP, _VP, _VP]),
    "mmfd_layernorm_bwd": (_I, [_I, _I64, _I64, _VP, _I64, _VP, _I64, _VP, _VP, _VP, _VP, _I64, _VP, _I64,
                                _VP, _VP, _F, _VP, _F, _VP, _U64, _VP, _I64, _VP]),
    "mmfd_seq_mean_fwd": (_I, [_I, _I64, _I64, _I64, _VP, _VP, _I64, _VP]),
    "mmfd_seq_mean_bwd": (_I, [_I, _I64, _I64, _I64, _VP, _I64, _VP, _VP]),
    "mmfd_xent_fwd_bwd": (_I, [_I, _I64, _I64, _VP, _VP, _VP, _I64, _VP, _I, _VP, _VP, _VP]),
    "mmfd_embed_ln_fwd": (_I, [_I, _I64, _I64, _I64, _VP, _VP, _VP, _VP, _VP, _VP, _VP, _F, _VP, _VP, _VP, _VP,
                               _F, _VP, _U64, _VP]),
    "mmfd_embed_bwd": (_I, [_I, _I64, _I64, _I64, _I64, _VP, _VP, _VP, _VP, _VP, _VP, _I64, _VP, _I64, _VP]),
    "mmfd_embed_bwd_workspace_bytes": (_I64, [_I64, _I64, _I64]),
    "mmfd_mask_to_bias": (_I, [_I64, _VP, _VP, _F, _VP]),
    "mmfd_embed_ln_fwd_ex": (_I, [_I, _I64, _I64, _I64, _VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP, _F, _VP, _VP, _VP, _VP,
                                  _F, _VP, _U64, _VP]),
    "mmfd_position_ids": (_I, [_I64, _I64, _VP, _I64, _VP, _VP]),
    "mmfd_conv_weight_prep": (_I, [_I, _I64, _I64, _I64, _I64, _I64, _VP, _VP, _VP, _VP, _VP, _F, _VP, _VP, _VP]),
    "mmfd_im2col_nhwc": (_I, [_I, _I64, _I64, _I64, _I64, _I, _I, _I, _I, _I64, _I64, _I64, _VP, _VP, _VP]),
    "mmfd_im2col_nchw": (_I, [_I, _I64, _I64, _I64, _I64, _I, _I, _I, _I, _I64, _I64, _I64, _VP, _VP, _VP]),
    "mmfd_maxpool_nhwc": (_I, [_I, _I64, _I64, _I64, _I64, _I, _I, _I, _I64, _I64, _VP, _VP, _VP]),
    "mmfd_global_avgpool": (_I, [_I, _I64, _I64, _I64, _VP, _VP, _VP]),
    "mmfd_rel_bias": (_I, [_I64, _I64, _I64, _VP, _VP, _VP, _VP]),
    "mmfd_deberta_rel_bias": (_I, [_I, _I64, _I64, _I64, _VP, _VP, _I64, _VP, _VP, _F, _VP, _VP]),
    "mmfd_mask_rows": (_I, [_I, _I64, _I64, _VP, _I64, _VP, _VP]),
    "mmfd_attn_fill_masked_rows": (_I, [_I, _I64, _I64, _I64, _I64, _VP, _I64, _I64, _VP, _I64, _I64, _VP, _VP]),
    "mmfd_patchify": (_I, [_I, _I64, _I64, _I64, _I64, _I64, _VP, _VP, _VP]),
    "mmfd_vit_tokens_fwd": (_I, [_I, _I64, _I64, _I64, _VP, _VP, _VP, _VP, _VP]),
    "mmfd_vit_tokens_bwd": (_I, [_I, _I64, _I64, _I64, _VP, _VP, _VP, _VP, _VP, _I64, _VP]),
    "mmfd_adamw": (_I, [_I, _VP, _I64, _F, _F, _F, _F, _F, _VP]),
    "mmfd_cast": (_I, [_I, _I, _I64, _VP, _VP, _VP]),
    "mmfd_zero": (_I, [_VP, _I64, _VP]),
    "mmfd_axpby": (_I, [_I, _I64, _F, _VP, _F, _VP, _VP, _VP]),
    "mmfd_dropout": (_I, [_I, _I64, _VP, _VP, _F, _VP, _U64, _VP]),
    "mmfd_seed_advance": (_I, [_VP, _VP]),
    "mmfd_act_bwd": (_I, [_I, _I64, _VP, _VP, _I, _F, _VP, _U64, _VP, _VP]),
    "mmfd_cosine_scores": (_I, [_I, _I64, _I64, _I64, _VP, _I64, _VP, _I64, _I, _F, _VP, _I64, _VP]),
    "mmfd_topk_workspace_bytes": (_I64, [_I64, _I64, _I64]),
    "mmfd_topk": (_I, [_I64, _I64, _VP, _I64, _I64, _VP, _VP, _VP, _I64, _VP]),
    "mmfd_resize_normalize": (_I, [_I64, _VP, _I64, _I64, _VP, _VP, _I64, _I64, ctypes.POINTER(ctypes.c_float),
                                   ctypes.POINTER(ctypes.c_float), _VP, _VP]),
    "mmfd_layernorm_fwd_res": (_I, [_I, _I64, _I64, _VP, _I64, _VP, _VP, _F, _VP, _I64, _VP, _I64, _VP, _VP, _VP]),
    "mmfd_row_gather": (_I, [_I64, _I64, _I64, _I64, _I64, _VP, _VP, _VP, _VP]),
    "mmfd_swin_cpb": (_I, [_I64, _I64, _VP, _VP, _VP, _VP, _VP, _VP]),
    "mmfd_swin_bias": (_I, [_I64, _I64, _I64, _VP, _VP, _VP, _VP, _VP]),
    "mmfd_swin_qk_norm": (_I, [_I, _I64, _I64, _I64, _VP, _I64, _VP, _F, _VP]),
}

_lib = None


def load(path: str = LIB_PATH):
    """Load libmmfd_hip.so (after torch, so the HIP runtime torch already loaded is reused)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise NativeLibraryError(f"{path} not found: run `python -c 'import __graft_entry__ as g; g.build()'`")
    try:
        lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    except OSError as e:  # pragma: no cover - depends on the box
        raise NativeLibraryError(f"cannot load {path}: {e}") from e
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.mmfd_version() != ABI_VERSION:
        raise NativeLibraryError(f"{path} implements ABI version {lib.mmfd_version()}, these bindings version "
                                 f"{ABI_VERSION}: rebuild (python -c 'import __graft_entry__ as g; g.build()')")
    if not os.path.exists(TORCH_LIB_PATH):
        raise NativeLibraryError(f"{TORCH_LIB_PATH} not found: run `python -c 'import __graft_entry__ as g; g.build()'`")
    try:
        torch.ops.load_library(TORCH_LIB_PATH)  # registers torch.ops.mmfd.* (needs libmmfd_hip.so loaded)
    except (OSError, RuntimeError) as e:  # pragma: no cover - depends on the box
        raise NativeLibraryError(f"cannot load {TORCH_LIB_PATH}: {e}") from e
    from . import ops  # noqa: F401  (fake kernels of the custom ops)
    _lib = lib
    return lib


def _ops():
    if _lib is None:
        load()
    return torch.ops.mmfd


def _salt(salt):
    """uint64 call-site salt -> the int64 of the op schema (same bits)"""
    salt = int(salt) & 0xFFFFFFFFFFFFFFFF
    return salt - (1 << 64) if salt >= (1 << 63) else salt


def lib():
    return _lib if _lib is not None else load()


def _check(rc: int, what: str):
    if rc != 0:
        msg = lib().mmfd_last_error_string().decode(errors="replace")
        raise RuntimeError(f"{what} failed (code {rc}): {msg}")


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def dtype_code(dt: torch.dtype) -> int:
    if dt == torch.float32:
        return F32
    if dt == torch.bfloat16:
        return BF16
    raise TypeError(f"unsupported dtype {dt} (fp32 / bf16)")


def _require_cuda(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("mmfd kernels need tensors on the GPU (HIP device)")


def salt_of(name: str) -> int:
    """Stable 64-bit call-site id for counter-based dropout."""
    b = name.encode()
    return (zlib.crc32(b) << 32) | zlib.crc32(b[::-1] + b"mmfd")


# ------------------------------------------------------------------------------------------------
# step seed (device resident so that captured graphs see it advance)
# ------------------------------------------------------------------------------------------------
class Seed:
    def __init__(self, value: int = 0, device=None):
        self.t = torch.tensor([value], dtype=torch.int64, device=device or "cuda")

    def ptr(self):
        return _ptr(self.t)

    def advance(self):
        _check(lib().mmfd_seed_advance(self.ptr(), _stream()), "seed_advance")

    def set(self, value: int):
        self.t.fill_(value)

    def fork(self):
        """Snapshot of the current value for one forward/backward pair (the kernels read the seed
        at launch time), then advance this seed for the next forward."""
        s = Seed.__new__(Seed)
        s.t = self.t.clone()
        self.advance()
        return s


# ------------------------------------------------------------------------------------------------
# GEMM
# ------------------------------------------------------------------------------------------------
def _ld(t: torch.Tensor) -> int:
    if t.dim() != 2 or t.stride(1) != 1:
        raise ValueError(f"operand must be a 2-D row-major view, got shape {tuple(t.shape)} strides {t.stride()}")
    return t.stride(0)


_PROBE = None


class GemmProbe:
    """Records HIP events around every MFMA-path GEMM launch while active (bench.py roofline):
    per kernel instantiation, the algorithmic FLOPs (2*M*N*K) and the launch's device time."""

    def __init__(self):
        self.records = []

    def __enter__(self):
        global _PROBE
        _PROBE = self
        return self

    def __exit__(self, *exc):
        global _PROBE
        _PROBE = None

    def summary(self):
        """per kernel instantiation {launches, flops, ms}"""
        torch.cuda.synchronize()
        out = {}
        for key, flops, e0, e1 in self.records:
            ms = e0.elapsed_time(e1)
            d = out.setdefault(key, {"launches": 0, "flops": 0, "ms": 0.0})
            d["launches"] += 1
            d["flops"] += flops
            d["ms"] += ms
        return out


def _x6(a):
    """whether mmfd_gemm runs this fp32 product on split bf16 operands: 0 no, 2 fused-plane kernel,
    1 segmented kernel (the library's own decision, mmfd_gemm_runs_split)"""
    return lib().mmfd_gemm_runs_split(ctypes.byref(a))


_FP32_MODE = None


def set_fp32_gemm_mode(mode):
    """fp32 GEMMs: 'split' (bf16 operand planes, six MFMA products, fp32 accumulation; the default)
    or 'native' (fp32 MFMA). Returns the previous mode name."""
    global _FP32_MODE
    code = {"native": 0, "split": 1}[mode]
    old = lib().mmfd_set_fp32_gemm_mode(code)
    _check(0 if old >= 0 else old, "mmfd_set_fp32_gemm_mode")
    _FP32_MODE = code
    return {0: "native", 1: "split"}[old]


def set_fp32_attn_mode(mode):
    """fp32 attention: 'split' (bf16 operand planes, six MFMA products per product, fp32
    accumulation; the default) or 'native' (fp32 MFMA). Returns the previous mode name."""
    code = {"native": 0, "split": 1}[mode]
    old = lib().mmfd_set_fp32_attn_mode(code)
    _check(0 if old >= 0 else old, "mmfd_set_fp32_attn_mode")
    return {0: "native", 1: "split"}[old]


_G4_MODES = {"off": 0, "on": 1, "gelu": 2}


def set_g4_mode(mode=None, kmax=None):
    """The four-wave bf16 forward GEMM (gemm_g4.hip): 'off', 'on' or 'gelu' (default: the FFN1 GELU
    epilogues too), and the largest K it takes. Returns the previous (mode, kmax); None leaves a
    setting as it is (A/B measurements and tests: set between launches, not per stream)."""
    old = lib().mmfd_set_g4_mode(-1 if mode is None else _G4_MODES[mode])
    _check(0 if old >= 0 else old, "mmfd_set_g4_mode")
    old_k = lib().mmfd_set_g4_kmax(0 if kmax is None else int(kmax))
    return {v: k for k, v in _G4_MODES.items()}[old], int(old_k)


def set_g4_persist(on=None):
    """the four-wave GEMM's persistent grid (default True) or one workgroup per tile; returns the
    previous setting (None only queries)"""
    old = lib().mmfd_set_g4_persist(-1 if on is None else int(bool(on)))
    _check(0 if old >= 0 else old, "mmfd_set_g4_persist")
    return bool(old)


def g4_takes(x2d, W, act, residual=None, dropout_p=0.0):
    """whether the four-wave GEMM runs x2d @ W^T (bf16 nn.Linear forward, contiguous operands) with
    this epilogue — mirrors mmfd_gemmx::g4_epi's shape / mode conditions; blocks.linear saves the
    GELU derivative (MMFD_ACT_GELU_D) only for products it takes (elsewhere GELU_D runs through a
    split-K slab and the reduce, which costs more than the backward's erf it saves)"""
    mode, kmax = g4_mode()
    if mode == "off" or x2d.dtype != torch.bfloat16 or W.dtype != torch.bfloat16:
        return False
    if act in (ACT_GELU, ACT_GELU_D) and mode != "gelu":
        return False
    (M, Kd), N = x2d.shape, W.shape[0]
    if M % 256 or N % 256 or Kd % 64 or Kd < 64 or Kd > kmax or residual is not None or dropout_p > 0:
        return False
    return _ld(x2d) % 8 == 0 and _ld(W) % 8 == 0 and x2d.data_ptr() % 16 == 0 and W.data_ptr() % 16 == 0


def g4_mode():
    """(mode, kmax) the library currently uses for the four-wave GEMM"""
    return set_g4_mode()


def fp32_gemm_mode():
    global _FP32_MODE
    if _FP32_MODE is None:  # the library's load-time default (env MMFD_FP32_GEMM)
        old = lib().mmfd_set_fp32_gemm_mode(1)
        lib().mmfd_set_fp32_gemm_mode(old)
        _FP32_MODE = old
    return _FP32_MODE


def _kernel_name(a, split):
    """the device kernel mmfd_gemm launches for these arguments (rocprof's demangled name)"""
    t = {F32: "float", BF16: "__bf16"}
    narrow = a.M >= 4096 and (a.N <= 128 or a.K < 64)  # gemm.hip use_g8
    g8 = not narrow and (a.dtype == BF16 or a.c_dtype == F32)
    if g8:  # 256x256 kernel; PRE = one prefetched bf16 epilogue operand stream; X6 = split operands
        streams = int(bool(a.ep.residual)) + int(a.ep.act in (ACT_GELU_BWD, ACT_RELU_BWD, ACT_MUL_AUX)) + int(a.beta != 0.0)
        pre = a.c_dtype == BF16 and streams == 1 and not split
        x6 = _x6(a)
        # the lean instantiations (no activation / dropout, or split-K slabs) keep the plain names
        lean = split or (a.ep.act == ACT_NONE and a.ep.dropout_p <= 0.0)
        if x6 == 2:  # gemm_x6f.hip launch_x6f (ext: GELU_D / MUL_AUX in the kernel's own epilogue)
            ext = not lean and a.ep.act in (ACT_GELU_D, ACT_MUL_AUX)
            base = f"gemm256_x6f{'' if lean else '_ext' if ext else '_act'}_kernel<{a.trans_a}, {a.trans_b}>"
        else:  # gemm256.h launch_g8_v
            base = (f"gemm256{'' if lean else '_act'}_kernel<{t[BF16 if x6 else a.dtype]}, {a.trans_a}, {a.trans_b}, "
                    f"{t[a.c_dtype]}, {'true' if pre else 'false'}, {'true' if x6 else 'false'}>")
    elif a.N <= 64 and not a.trans_b:  # gemm.hip launch_mfma: the 256x64 tile
        base = f"gemm_mfma_n64_kernel<{t[a.dtype]}, {a.trans_a}, {t[a.c_dtype]}>"
    else:
        base = f"gemm_mfma_kernel<{t[a.dtype]}, {a.trans_a}, {a.trans_b}, {t[a.c_dtype]}>"
    return base + (" (split-K)" if split else "")


def gemm(A, B, *, trans_a=False, trans_b=False, out=None, out_dtype=None, alpha=1.0, beta=0.0, bias=None,
         residual=None, act=ACT_NONE, aux=None, dropout_p=0.0, seed=None, salt=0, splits=0, a_rowsum=None,
         a_rowsum_beta=0.0, residual_first=False, a_planes=None, b_planes=None, out_planes=None, write_out=True):
    """C = epilogue(alpha * op(A) @ op(B)) with op(A) = A or A^T ([M,K]) and op(B) = B^T ([N,K] stored,
    nn.Linear weight) when trans_b=False, else B ([K,N] stored). `a_rowsum` (fp32 [M]) additionally
    receives a_rowsum_beta * a_rowsum + sum_k op(A)[m, k] (bias gradient of a weight-gradient GEMM).
    `a_planes` / `b_planes`: split3() of the stored fp32 A / B, reused by the split-operand fp32 GEMM.
    `out_planes` (bf16 [3, M, N], fp32 output only): the output's split planes, written by the
    epilogue; with write_out=False instead of `out` (which then only carries the shape and stays
    unwritten — only for outputs read by split-operand GEMMs alone, see x6_ok)."""
    _require_cuda(A, B, out, bias, residual, aux)
    if A.dtype != B.dtype:
        raise TypeError(f"gemm operands must share a dtype ({A.dtype} vs {B.dtype})")
    if trans_a:
        K, M = A.shape
    else:
        M, K = A.shape
    if trans_b:
        K2, N = B.shape
    else:
        N, K2 = B.shape
    if K != K2:
        raise ValueError(f"gemm inner dims differ: {K} vs {K2}")
    if out is None:
        out = torch.empty((M, N), device=A.device, dtype=out_dtype or A.dtype)
    if tuple(out.shape) != (M, N):
        raise ValueError(f"gemm out shape {tuple(out.shape)} != {(M, N)}")
    if bias is not None and (bias.dtype != torch.float32 or bias.numel() != N or not bias.is_contiguous()):
        raise ValueError("bias must be a contiguous fp32 vector of length N")
    for t in (residual, aux):
        if t is not None and (t.dtype != out.dtype or tuple(t.shape) != (M, N)):
            raise ValueError("residual/aux must match the output shape and dtype")
    if dropout_p > 0 and seed is None:
        raise ValueError("dropout needs a Seed")
    if a_rowsum is not None:
        if a_rowsum.dtype != torch.float32 or a_rowsum.numel() != M or not a_rowsum.is_contiguous():
            raise ValueError("a_rowsum must be a contiguous fp32 vector of length M")
        _require_cuda(a_rowsum)
    probe = _PROBE
    rec = probe is not None and M >= 16 and N >= 16 and K >= 16 and not torch.cuda.is_current_stream_capturing()
    if rec:
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record()
    _ops().gemm(A, B, bool(trans_a), bool(trans_b), out, float(alpha), float(beta), bias, residual,
                bool(residual_first), int(act), aux, float(dropout_p), seed.t if seed is not None else None,
                _salt(salt), int(splits), a_rowsum, float(a_rowsum_beta), a_planes, b_planes, out_planes,
                bool(write_out), bool(getattr(A, "_mmfd_planes_only", False)),
                bool(getattr(B, "_mmfd_planes_only", False)))
    if not write_out:  # the fp32 output stays unwritten: only its planes may be read (checked in mmfd_gemm)
        out._mmfd_planes_only = True
    if rec:
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        probe.records.append((_probe_name(A, B, out, trans_a, trans_b, residual, act, beta, splits, alpha=alpha,
                                          residual_first=residual_first, dropout_p=dropout_p, a_rowsum=a_rowsum,
                                          aux=aux, bias=bias), 2 * M * N * K, e0, e1))
    return out


def _g4_mode(A, B, out, trans_a, trans_b, residual, act, beta, splits, alpha, residual_first, dropout_p, a_rowsum,
             aux, bias):
    """the four-wave kernel's epilogue mode for this product, or None (mirrors mmfd_gemmx::launch_g4;
    GemmProbe bookkeeping only)"""
    g4, kmax = g4_mode()  # the library's own switches (mmfd_set_g4_mode)
    if g4 == "off" or trans_a or trans_b or splits > 1 or a_rowsum is not None:
        return None
    if A.dtype != torch.bfloat16 or out.dtype != torch.bfloat16 or alpha != 1.0 or beta != 0.0:
        return None
    M, K = A.shape
    N = B.shape[0]
    if M % 256 or N % 256 or K % 64 or K < 64 or K > kmax:
        return None
    ts = [t for t in (A, B, out, residual, aux, bias) if t is not None]
    if any(t.data_ptr() % 16 for t in ts) or any(_ld(t) % 8 for t in (A, B, out, residual, aux) if t is not None):
        return None
    if act == ACT_NONE and residual is None and dropout_p <= 0:
        return 0
    if act == ACT_NONE and residual is not None and not residual_first:
        return 2 if dropout_p > 0 else 1
    if act == ACT_GELU and residual is None and dropout_p <= 0 and g4 == "gelu":
        return 3
    if act == ACT_GELU_BWD and aux is not None and residual is None and dropout_p <= 0:
        return 4
    if act == ACT_GELU_D and residual is None and dropout_p <= 0 and g4 == "gelu":
        return 5
    if act == ACT_MUL_AUX and aux is not None and residual is None and dropout_p <= 0:
        return 6
    return None


def _probe_name(A, B, out, trans_a, trans_b, residual, act, beta, splits, alpha=1.0, residual_first=False,
                dropout_p=0.0, a_rowsum=None, aux=None, bias=None):
    """the kernel instantiation mmfd_gemm picks (GemmProbe bookkeeping only)"""
    g4 = _g4_mode(A, B, out, trans_a, trans_b, residual, act, beta, splits, alpha, residual_first, dropout_p,
                  a_rowsum, aux, bias)
    if g4 is not None:
        return f"gemm_g4_kernel<{g4}>"
    M, K = (A.shape[1], A.shape[0]) if trans_a else A.shape
    N = B.shape[1] if trans_b else B.shape[0]
    a = GemmArgs()
    a.dtype, a.c_dtype = dtype_code(A.dtype), dtype_code(out.dtype)
    a.trans_a, a.trans_b = int(bool(trans_a)), int(bool(trans_b))
    a.M, a.N, a.K = M, N, K
    a.A, a.lda, a.B, a.ldb = A.data_ptr(), _ld(A), B.data_ptr(), _ld(B)
    a.C, a.ldc = out.data_ptr(), _ld(out)
    a.beta, a.splits = float(beta), int(splits)
    if residual is not None:
        a.ep.residual, a.ep.ldr = residual.data_ptr(), _ld(residual)
    a.ep.act = int(act)
    return _kernel_name(a, lib().mmfd_gemm_splits(ctypes.byref(a)) > 1)


def split3(x, out=None):
    """fp32 [rows, cols] (row-major view, cols % 8 == 0) -> bf16 planes [3, rows, cols]: hi = bf16(x),
    mid = bf16(x - hi), lo = bf16(x - hi - mid) — the operand form of the split-operand fp32 GEMM"""
    _require_cuda(x)
    if x.dtype != torch.float32 or x.dim() != 2:
        raise TypeError("split3 takes a 2-D fp32 tensor")
    if out is None:
        out = torch.empty((3, x.shape[0], x.shape[1]), device=x.device, dtype=torch.bfloat16)
    _ops().split3(x, out)
    return out


def x6_ok(M, N, K, trans_a=False, trans_b=False):
    """whether mmfd_gemm runs this fp32 product (contiguous operands) on split operands — asked of
    the library itself (mmfd_gemm_runs_split: x6_plan + use_g8 + mfma_ok, every env switch
    included), so a producer never skips an fp32 output that a consumer would then read"""
    if fp32_gemm_mode() != 1 or min(M, N, K) < 1:
        return False
    a = GemmArgs()
    a.dtype = a.c_dtype = F32
    a.trans_a, a.trans_b = int(bool(trans_a)), int(bool(trans_b))
    a.M, a.N, a.K = int(M), int(N), int(K)
    a.A = a.B = a.C = 1 << 20  # placeholder 16-B aligned pointers: only the shapes are inspected
    a.lda = M if trans_a else K
    a.ldb = N if trans_b else K
    a.ldc = N
    return lib().mmfd_gemm_runs_split(ctypes.byref(a)) != 0


def split_eligible(x):
    """whether GEMMs on fp32 operand `x` run on split planes (mode split, 16-B plane rows)"""
    return (x is not None and x.dtype == torch.float32 and x.dim() == 2 and x.shape[1] % 8 == 0
            and x.stride(1) == 1 and fp32_gemm_mode() == 1 and 6 * x.numel() < (1 << 31) - 4096)


def colsum(X, out=None, beta=0.0):
    _require_cuda(X)
    M, N = X.shape
    if out is None:
        out = torch.empty(N, device=X.device, dtype=torch.float32)
    nparts = max(1, min(256, M // 64))
    ws = torch.empty(nparts * N, device=X.device, dtype=torch.float32)
    _check(lib().mmfd_colsum(dtype_code(X.dtype), M, N, _ptr(X), _ld(X), _ptr(out), float(beta), _ptr(ws),
                             ws.numel() * 4, _stream()), "mmfd_colsum")
    return out


def linear(x, w, b=None, **kw):
    """y = x @ w^T + b over the last dim (x: [..., K], w: [N, K])."""
    shp = x.shape
    y = gemm(x.reshape(-1, shp[-1]), w, bias=b, **kw)
    return y.reshape(*shp[:-1], w.shape[0])


# ------------------------------------------------------------------------------------------------
# attention
# ------------------------------------------------------------------------------------------------
def _head_view(t, H, D):
    """t: [B, L, >= H*D] view with unit stride on the last dim -> (ptr, s_b, s_t)."""
    if t.dim() != 3 or t.stride(2) != 1:
        raise ValueError("attention operands must be [B, L, H*D] views with a contiguous last dim")
    return t.data_ptr(), t.stride(0), t.stride(1)


def drop_mask_buffer(B, H, Lq, Lk, device):
    """the dropout keep-bitmask of one attention call (include/mmfd.h mmfd_attn_args.drop_mask): int32
    words [B*H*Lq*ceil(Lk/32)], written by attn_fwd and read by attn_bwd instead of re-hashing"""
    return torch.empty(B * H * Lq * ((Lk + 31) // 32), device=device, dtype=torch.int32)


def attn_fwd(q, k, v, H, *, out=None, scale=None, key_bias=None, rel_bias=None, dropout_p=0.0, seed=None, salt=0,
             cos_logit_scale=None, cos_max_log=0.0, o_planes=None, drop_mask=None):
    """q: [B, Lq, H*D], k/v: [B, Lk, H*D] (views into fused QKV buffers are fine).
    cos_logit_scale (fp32 [H], bf16 only): Swinv2 cosine attention, q/k normalised in the kernel.
    drop_mask (drop_mask_buffer, with dropout_p > 0): receives the keep-bitmask for attn_bwd.
    Returns (o [B, Lq, H*D], lse [B, H, Lq] fp32)."""
    _require_cuda(q, k, v)
    B, Lq, HD = q.shape
    Lk = k.shape[1]
    D = HD // H
    if out is None:
        out = torch.empty((B, Lq, H * D), device=q.device, dtype=q.dtype)
    lse = torch.empty((B, H, Lq), device=q.device, dtype=torch.float32)
    _head_view(q, H, D), _head_view(k, H, D), _head_view(v, H, D), _head_view(out, H, D)
    rb, rb_sb, rb_mod = _rel_bias_args(rel_bias, B, H, Lq, Lk)
    if cos_logit_scale is not None and (cos_logit_scale.dtype != torch.float32 or not cos_logit_scale.is_contiguous()):
        raise ValueError("cos_logit_scale must be a contiguous fp32 tensor of H values")
    _ops().attn_fwd(q, k, v, out, lse, int(H), float(scale if scale is not None else D ** -0.5), key_bias,
                    rel_bias if rb is not None else None, int(rb_sb), int(rb_mod), float(dropout_p),
                    seed.t if seed is not None else None, _salt(salt), cos_logit_scale, float(cos_max_log), o_planes,
                    drop_mask if dropout_p > 0 else None)
    return out, lse


def _rel_bias_args(rel_bias, B, H, Lq, Lk):
    """(pointer, batch stride, batch modulus) for an additive fp32 bias shared by the batch
    ([H, Lq, Lk], MPNet), per batch row ([B, H, Lq, Lk], DeBERTa) or repeating every M batch rows
    ([M, H, Lq, Lk] with B % M == 0: Swinv2 shifted-window masks, batch = images x M windows)"""
    if rel_bias is None:
        return None, 0, 0
    if rel_bias.dtype != torch.float32 or not rel_bias.is_contiguous():
        raise ValueError("rel_bias must be a contiguous fp32 tensor")
    if tuple(rel_bias.shape) == (H, Lq, Lk):
        return rel_bias.data_ptr(), 0, 0
    if tuple(rel_bias.shape) == (B, H, Lq, Lk):
        return rel_bias.data_ptr(), H * Lq * Lk, 0
    if rel_bias.dim() == 4 and tuple(rel_bias.shape[1:]) == (H, Lq, Lk) and B % rel_bias.shape[0] == 0:
        return rel_bias.data_ptr(), H * Lq * Lk, rel_bias.shape[0]
    raise ValueError(f"rel_bias shape {tuple(rel_bias.shape)} is neither [H,Lq,Lk] nor [M,H,Lq,Lk] with B % M == 0")


def deberta_rel_bias(c2p, p2c, c2p_idx, p2c_idx, B, L, inv_scale, out=None):
    """DeBERTa c2p + p2c bias [B, H, L, L] fp32 from the per-head position scores c2p / p2c
    ([H, B*L, ld]) and the clamped log-bucket indices (int32 [L, L])."""
    _require_cuda(c2p, p2c, c2p_idx, p2c_idx)
    H, _, ld = c2p.shape
    out = out if out is not None else torch.empty((B, H, L, L), device=c2p.device, dtype=torch.float32)
    _check(lib().mmfd_deberta_rel_bias(dtype_code(c2p.dtype), B, H, L, _ptr(c2p), _ptr(p2c), ld, _ptr(c2p_idx),
                                       _ptr(p2c_idx), float(inv_scale), _ptr(out), _stream()), "mmfd_deberta_rel_bias")
    return out


def mask_rows(x2d, mask):
    """x[r, :] = 0 where mask[r] == 0 (in place)"""
    _require_cuda(x2d, mask)
    m = mask.reshape(-1).to(torch.int64).contiguous()
    _check(lib().mmfd_mask_rows(dtype_code(x2d.dtype), x2d.shape[0], x2d.shape[1], _ptr(x2d), _ld(x2d), _ptr(m),
                                _stream()), "mmfd_mask_rows")
    return x2d


def attn_fill_masked_rows(v, o, H, mask):
    """o rows of fully masked queries (mask[b, i] == 0) = mean of v over all keys (in place)"""
    _require_cuda(v, o, mask)
    B, L, HD = v.shape
    Dh = HD // H
    m = mask.to(torch.int64).contiguous()
    vp, vsb, vst = _head_view(v, H, Dh)
    op, osb, ost = _head_view(o, H, Dh)
    _check(lib().mmfd_attn_fill_masked_rows(dtype_code(v.dtype), B, H, L, Dh, vp, vsb, vst, op, osb, ost, _ptr(m),
                                            _stream()), "mmfd_attn_fill_masked_rows")
    return o


def attn_bwd(q, k, v, o, lse, dout, H, *, dq=None, dk=None, dv=None, scale=None, key_bias=None, rel_bias=None,
             dropout_p=0.0, seed=None, salt=0, accumulate_dq=False, accumulate_dkv=False, dqkv_planes=None,
             planes_only=False, drop_mask=None):
    """dq, dk, dv (views of one packed [B, L, 3*H*D] buffer when `dqkv_planes` is given: bf16
    [3, B*L, 3*H*D] split planes of that buffer, written by the kernels; planes_only skips the
    fp32 stores — for a gradient read only by split-operand GEMMs, see x6_ok)"""
    _require_cuda(q, k, v, o, lse, dout)
    B, Lq, HD = q.shape
    Lk = k.shape[1]
    D = HD // H
    dq = dq if dq is not None else torch.empty_like(q, memory_format=torch.contiguous_format)
    dk = dk if dk is not None else torch.empty((B, Lk, HD), device=q.device, dtype=q.dtype)
    dv = dv if dv is not None else torch.empty((B, Lk, HD), device=q.device, dtype=q.dtype)
    for t in (q, k, v, o, dout, dq, dk, dv):
        _head_view(t, H, D)
    rb, rb_sb, rb_mod = _rel_bias_args(rel_bias, B, H, Lq, Lk)
    _ops().attn_bwd(q, k, v, o, lse, dout, dq, dk, dv, int(H), float(scale if scale is not None else D ** -0.5),
                    key_bias, rel_bias if rb is not None else None, int(rb_sb), int(rb_mod), float(dropout_p),
                    seed.t if seed is not None else None, _salt(salt), bool(accumulate_dq), bool(accumulate_dkv),
                    dqkv_planes, bool(planes_only), drop_mask if dropout_p > 0 else None)
    return dq, dk, dv


# ------------------------------------------------------------------------------------------------
# LayerNorm
# ------------------------------------------------------------------------------------------------
def layernorm_fwd(x2d, gamma, beta, eps, out=None, planes=None):
    """y = LayerNorm(x); `planes` (bf16 [3, R, W], fp32 x only): the output's split3 planes, written
    in the same pass"""
    _require_cuda(x2d, gamma, beta)
    R, W = x2d.shape
    y = out if out is not None else torch.empty((R, W), device=x2d.device, dtype=x2d.dtype)
    mean = torch.empty(R, device=x2d.device, dtype=torch.float32)
    rstd = torch.empty(R, device=x2d.device, dtype=torch.float32)
    _ops().layernorm_fwd(x2d, gamma, beta, float(eps), y, mean, rstd, planes)
    return y, mean, rstd


def layernorm_fwd_res(x2d, gamma, beta, eps, res, out=None, stats=False):
    """y = res + LN(x) (Swinv2 res-post-norm); returns y (and mean, rstd when stats=True)"""
    _require_cuda(x2d, gamma, beta, res)
    R, W = x2d.shape
    if tuple(res.shape) != (R, W) or res.dtype != x2d.dtype:
        raise ValueError("layernorm_fwd_res: residual must match x in shape and dtype")
    y = out if out is not None else torch.empty((R, W), device=x2d.device, dtype=x2d.dtype)
    mean = torch.empty(R, device=x2d.device, dtype=torch.float32) if stats else None
    rstd = torch.empty(R, device=x2d.device, dtype=torch.float32) if stats else None
    _check(lib().mmfd_layernorm_fwd_res(dtype_code(x2d.dtype), R, W, _ptr(x2d), _ld(x2d), _ptr(gamma), _ptr(beta),
                                        float(eps), _ptr(res), _ld(res), _ptr(y), _ld(y),
                                        _ptr(mean) if stats else None, _ptr(rstd) if stats else None, _stream()),
           "mmfd_layernorm_fwd_res")
    return (y, mean, rstd) if stats else y


def layernorm_bwd(dy, x, gamma, mean, rstd, *, dx=None, dx_add=None, dgamma=None, dbeta=None, beta_acc=0.0,
                  dx_drop=None, dropout_p=0.0, seed=None, salt=0, planes=None):
    """`planes` (bf16 [3, R, W], fp32 only): split planes of the gradient the next GEMMs read —
    dx_drop when given, else dx — written by the same kernel"""
    _require_cuda(dy, x, gamma, mean, rstd)
    R, W = dy.shape
    dx = dx if dx is not None else torch.empty((R, W), device=dy.device, dtype=dy.dtype)
    _ops().layernorm_bwd(dy, x, gamma, mean, rstd, dx, dx_add, dgamma, dbeta, float(beta_acc), dx_drop,
                         float(dropout_p), seed.t if seed is not None else None, _salt(salt), planes)
    return dx


# ------------------------------------------------------------------------------------------------
# misc
# ------------------------------------------------------------------------------------------------
def seq_mean_fwd(x, out=None):
    B, L, D = x.shape
    out = out if out is not None else torch.empty((B, D), device=x.device, dtype=x.dtype)
    _ops().seq_mean_fwd(x if x.is_contiguous() else x.contiguous(), out)
    return out


def seq_mean_bwd(dout, L, dx=None):
    B, D = dout.shape
    dx = dx if dx is not None else torch.empty((B, L, D), device=dout.device, dtype=dout.dtype)
    _ops().seq_mean_bwd(dout, dx)
    return dx


def xent_fwd_bwd(logits, labels, want_grad=True, dloss_scale=None, cols=None, n_slots=None):
    """logits: list of [B, C] fp32 tensors (present paths), labels: int64 [B, n_cols] (or [B]);
    cols: label column of each path (the reference's path index, train.py:165; default 0..n-1).
    Returns (loss [n_slots] fp32 device tensor: total, then one slot per label column (0 for
    columns without a present path), list of dlogits or None)."""
    n = len(logits)
    B, C = logits[0].shape
    dev = logits[0].device
    cols = list(range(n)) if cols is None else [int(c) for c in cols]
    if len(cols) != n:
        raise ValueError("xent: one label column per path")
    n_slots = n_slots or 1 + max(cols) + 1
    logits = [l.contiguous().float() for l in logits]
    labels = labels.contiguous()
    ld = labels.stride(0) if labels.dim() > 1 else 1
    if max(cols) >= (labels.shape[1] if labels.dim() > 1 else 1):
        raise ValueError(f"xent: label column {max(cols)} outside labels {tuple(labels.shape)}")
    del ld
    loss = torch.empty(n_slots, device=dev, dtype=torch.float32)
    dl = [torch.empty_like(l) for l in logits] if want_grad else None
    _ops().xent(logits, cols, labels, loss, dl if want_grad else [], dloss_scale)
    return loss, dl


def cast(x, dtype, out=None):
    if out is None:
        out = torch.empty(x.shape, device=x.device, dtype=dtype)
    elif out.dtype != dtype or out.numel() != x.numel() or not out.is_contiguous():
        raise ValueError("cast: out must be a contiguous tensor of the target dtype and size")
    if x.numel():
        _ops().cast(x if x.is_contiguous() else x.contiguous(), out)
    return out


def transpose(x, out=None):
    """out = x^T as a contiguous [cols, rows] tensor (fp32 / bf16, mmfd_transpose)"""
    _require_cuda(x)
    if x.dim() != 2:
        raise ValueError("transpose takes a 2-D tensor")
    rows, cols = x.shape
    if out is None:
        out = torch.empty((cols, rows), device=x.device, dtype=x.dtype)
    if out.dtype != x.dtype or tuple(out.shape) != (cols, rows):
        raise ValueError("transpose: out must be [cols, rows] of the input dtype")
    _check(lib().mmfd_transpose(dtype_code(x.dtype), rows, cols, _ptr(x), _ld(x), _ptr(out), _ld(out), _stream()),
           "mmfd_transpose")
    return out


def zero_(t):
    """t[...] = 0 in place (a contiguous tensor) with mmfd_zero (a zero-fill kernel on the current stream)"""
    if not t.is_contiguous():
        raise ValueError("zero_: contiguous tensors only")
    if t.numel():
        _check(lib().mmfd_zero(_ptr(t), t.numel() * t.element_size(), _stream()), "mmfd_zero")
    return t


def zeros(shape, dtype=torch.float32, device="cuda"):
    """torch.empty + mmfd_zero"""
    return zero_(torch.empty(shape, dtype=dtype, device=device))


def axpby(a, x, b=0.0, y=None, out=None):
    out = out if out is not None else torch.empty_like(x)
    _check(lib().mmfd_axpby(dtype_code(x.dtype), x.numel(), float(a), _ptr(x), float(b), _ptr(y), _ptr(out),
                            _stream()), "mmfd_axpby")
    return out


def dropout(x, p, seed, salt, out=None):
    out = out if out is not None else torch.empty_like(x)
    _check(lib().mmfd_dropout(dtype_code(x.dtype), x.numel(), _ptr(x), _ptr(out), float(p), seed.ptr(),
                              int(salt) & 0xFFFFFFFFFFFFFFFF, _stream()), "mmfd_dropout")
    return out


def act_bwd(dy, aux, act, dropout_p=0.0, seed=None, salt=0, out=None):
    out = out if out is not None else torch.empty_like(dy)
    _check(lib().mmfd_act_bwd(dtype_code(dy.dtype), dy.numel(), _ptr(dy), _ptr(aux), int(act), float(dropout_p),
                              seed.ptr() if seed is not None else None, int(salt) & 0xFFFFFFFFFFFFFFFF, _ptr(out),
                              _stream()), "mmfd_act_bwd")
    return out


def mask_to_bias(mask, neg=None):
    neg = torch.finfo(torch.float32).min if neg is None else neg
    m = mask.to(torch.int64).contiguous()
    out = torch.empty(m.shape, device=m.device, dtype=torch.float32)
    _check(lib().mmfd_mask_to_bias(m.numel(), _ptr(m), _ptr(out), float(neg), _stream()), "mmfd_mask_to_bias")
    return out


def embed_ln_fwd(ids, tts, word, pos, typ, gamma, beta, eps, dtype, dropout_p=0.0, seed=None, salt=0):
    B, L = ids.shape
    D = word.shape[1]
    dev = ids.device
    s = torch.empty((B * L, D), device=dev, dtype=dtype)
    y = torch.empty((B * L, D), device=dev, dtype=dtype)
    mean = torch.empty(B * L, device=dev, dtype=torch.float32)
    rstd = torch.empty(B * L, device=dev, dtype=torch.float32)
    _check(lib().mmfd_embed_ln_fwd(dtype_code(dtype), B, L, D, _ptr(ids.contiguous()),
                                   _ptr(tts.contiguous()) if tts is not None else None, _ptr(word), _ptr(pos),
                                   _ptr(typ), _ptr(gamma), _ptr(beta), float(eps), _ptr(s), _ptr(y), _ptr(mean),
                                   _ptr(rstd), float(dropout_p), seed.ptr() if seed is not None else None,
                                   int(salt) & 0xFFFFFFFFFFFFFFFF, _stream()), "mmfd_embed_ln_fwd")
    return s, y, mean, rstd


def embed_ln_infer(ids, pos_ids, word, pos, gamma, beta, eps, dtype, tts=None, typ=None):
    """inference embeddings: y = LN(word[id] + pos[pos_id] (+ type[tt])), nothing saved"""
    B, L = ids.shape
    D = word.shape[1]
    y = torch.empty((B * L, D), device=ids.device, dtype=dtype)
    _check(lib().mmfd_embed_ln_fwd_ex(dtype_code(dtype), B, L, D, _ptr(ids.contiguous()),
                                      _ptr(pos_ids.contiguous()) if pos_ids is not None else None,
                                      _ptr(tts.contiguous()) if tts is not None else None, _ptr(word), _ptr(pos),
                                      _ptr(typ) if typ is not None else None, _ptr(gamma), _ptr(beta), float(eps),
                                      None, _ptr(y), None, None, 0.0, None, 0, _stream()), "mmfd_embed_ln_fwd_ex")
    return y


def position_ids(ids, padding_idx):
    ids = ids.contiguous()
    out = torch.empty_like(ids)
    _check(lib().mmfd_position_ids(ids.shape[0], ids.shape[1], _ptr(ids), int(padding_idx), _ptr(out), _stream()),
           "mmfd_position_ids")
    return out


def rel_bias(bucket, table):
    """bucket int32 [Lq, Lk] (device), table fp32 [nb, H] -> fp32 [H, Lq, Lk]"""
    Lq, Lk = bucket.shape
    H = table.shape[1]
    out = torch.empty((H, Lq, Lk), device=table.device, dtype=torch.float32)
    _check(lib().mmfd_rel_bias(H, Lq, Lk, _ptr(bucket.contiguous()), _ptr(table.contiguous()), _ptr(out), _stream()),
           "mmfd_rel_bias")
    return out


# ---- convolution support (ResNet50 extractor) ------------------------------------------------
def conv_weight_prep(w, dtype, Kpad=None, bn=None, eps=1e-5):
    """fp32 conv weight [Cout, Cin, KH, KW] (+ BatchNorm (gamma, beta, mean, var)) -> GEMM weight
    [Cout, Kpad] in dtype with (kh, kw, c) column order, and the folded fp32 bias [Cout]."""
    Cout, Cin, KH, KW = w.shape
    Kpad = Kpad or KH * KW * Cin
    ow = torch.empty((Cout, Kpad), device=w.device, dtype=dtype)
    ob = torch.empty(Cout, device=w.device, dtype=torch.float32)
    g, b, m, v = bn if bn is not None else (None, None, None, None)
    _check(lib().mmfd_conv_weight_prep(dtype_code(dtype), Cout, Cin, KH, KW, Kpad, _ptr(w.contiguous()),
                                       _ptr(g) if g is not None else None, _ptr(b) if b is not None else None,
                                       _ptr(m) if m is not None else None, _ptr(v) if v is not None else None,
                                       float(eps), _ptr(ow), _ptr(ob), _stream()), "mmfd_conv_weight_prep")
    return ow, ob


def im2col_nhwc(x, N, H, W, C, k, stride, pad, Kpad=None):
    Ho, Wo = (H + 2 * pad - k) // stride + 1, (W + 2 * pad - k) // stride + 1
    Kpad = Kpad or k * k * C
    out = torch.empty((N * Ho * Wo, Kpad), device=x.device, dtype=x.dtype)
    _check(lib().mmfd_im2col_nhwc(dtype_code(x.dtype), N, H, W, C, k, k, stride, pad, Ho, Wo, Kpad, _ptr(x), _ptr(out),
                                  _stream()), "mmfd_im2col_nhwc")
    return out, Ho, Wo


def im2col_nchw(x, k, stride, pad, Kpad, dtype):
    N, C, H, W = x.shape
    Ho, Wo = (H + 2 * pad - k) // stride + 1, (W + 2 * pad - k) // stride + 1
    out = torch.empty((N * Ho * Wo, Kpad), device=x.device, dtype=dtype)
    _check(lib().mmfd_im2col_nchw(dtype_code(dtype), N, C, H, W, k, k, stride, pad, Ho, Wo, Kpad,
                                  _ptr(x.contiguous()), _ptr(out), _stream()), "mmfd_im2col_nchw")
    return out, Ho, Wo


def conv_implicit_ok(dtype, C):
    """whether a convolution over C input channels can run as an implicit GEMM (conv2d_nhwc): a
    K-tile / split-operand K-step (64 bf16 / 32 fp32 channels) must not straddle two filter taps"""
    return C % (64 if dtype == torch.bfloat16 else 32) == 0


def conv2d_nhwc(x, N, H, W, C, w, k, stride, pad, bias=None, act=ACT_NONE, residual=None, residual_first=False,
                x_planes=None):
    """Implicit-GEMM convolution (mmfd_gemm_args.conv): x = the NHWC activation as rows [N*H*W, C],
    w = the folded GEMM weight [Cout, k*k*C] with (kh, kw, c) columns (conv_weight_prep), output
    rows [N*Ho*Wo, Cout] = epilogue(conv(x)) — the same products, in the same K order, as
    gemm(im2col_nhwc(x), w) without the im2col matrix (im2im_retrieval.py:14-17, 29-36).
    `x_planes`: split3(x), reused by the split-operand fp32 path when given. Returns (y, Ho, Wo)."""
    _require_cuda(x, w, bias, residual)
    if x.dtype != w.dtype:
        raise TypeError(f"conv operands must share a dtype ({x.dtype} vs {w.dtype})")
    if not conv_implicit_ok(x.dtype, C) or tuple(x.shape) != (N * H * W, C) or not x.is_contiguous():
        raise ValueError(f"conv2d_nhwc: x must be contiguous [N*H*W, C] with C % {64 if x.dtype == torch.bfloat16 else 32} == 0")
    Cout, Kw = w.shape
    if Kw != k * k * C or not w.is_contiguous():
        raise ValueError(f"conv2d_nhwc: w must be contiguous [Cout, {k * k * C}], got {tuple(w.shape)}")
    Ho, Wo = (H + 2 * pad - k) // stride + 1, (W + 2 * pad - k) // stride + 1
    M, K = N * Ho * Wo, k * k * C
    out = torch.empty((M, Cout), device=x.device, dtype=x.dtype)
    if bias is not None and (bias.dtype != torch.float32 or bias.numel() != Cout or not bias.is_contiguous()):
        raise ValueError("bias must be a contiguous fp32 vector of length Cout")
    if residual is not None and (residual.dtype != out.dtype or tuple(residual.shape) != (M, Cout)):
        raise ValueError("residual must match the output shape and dtype")
    g = ConvGeomArgs(N=N, H=H, W=W, C=C, KH=k, KW=k, stride=stride, pad=pad, Ho=Ho, Wo=Wo)
    a = GemmArgs()
    a.dtype = a.c_dtype = dtype_code(x.dtype)
    a.M, a.N, a.K = M, Cout, K
    a.A, a.lda, a.B, a.ldb = x.data_ptr(), C, w.data_ptr(), K
    a.C, a.ldc = out.data_ptr(), Cout
    a.alpha = 1.0
    if bias is not None:
        a.ep.bias = bias.data_ptr()
    if residual is not None:
        a.ep.residual, a.ep.ldr = residual.data_ptr(), _ld(residual)
        a.ep.residual_first = int(bool(residual_first))
    a.ep.act = int(act)
    if x_planes is not None:
        if x_planes.dtype != torch.bfloat16 or tuple(x_planes.shape) != (3, N * H * W, C) or not x_planes.is_contiguous():
            raise ValueError("x_planes must be split3(x): contiguous bf16 [3, N*H*W, C]")
        a.a_planes = x_planes.data_ptr()
    a.conv = ctypes.addressof(g)
    need = lib().mmfd_gemm_workspace_bytes(ctypes.byref(a))
    if need < 0:
        raise RuntimeError("mmfd_gemm_workspace_bytes failed: " + lib().mmfd_last_error_string().decode())
    ws = torch.empty(max(need, 1), device=x.device, dtype=torch.uint8) if need > 0 else None
    if ws is not None:
        a.workspace, a.workspace_bytes = ws.data_ptr(), need
    probe = _PROBE
    rec = probe is not None and not torch.cuda.is_current_stream_capturing()
    if rec:
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record()
    _check(lib().mmfd_gemm(ctypes.byref(a), _stream()), "mmfd_gemm (conv)")
    if rec:
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        split = lib().mmfd_gemm_splits(ctypes.byref(a)) > 1
        tn = "__bf16" if x.dtype == torch.bfloat16 else "float"
        name = ("conv_x6f_kernel" if _x6(a) == 2 else
                f"conv_mfma_kernel<{tn}, {tn}, {64 if Cout <= 64 else 128}>") + (" (split-K)" if split else "")
        probe.records.append((name, 2 * M * Cout * K, e0, e1))
    return out, Ho, Wo


def maxpool_nhwc(x, N, H, W, C, k=3, stride=2, pad=1):
    Ho, Wo = (H + 2 * pad - k) // stride + 1, (W + 2 * pad - k) // stride + 1
    out = torch.empty((N * Ho * Wo, C), device=x.device, dtype=x.dtype)
    _check(lib().mmfd_maxpool_nhwc(dtype_code(x.dtype), N, H, W, C, k, stride, pad, Ho, Wo, _ptr(x), _ptr(out),
                                   _stream()), "mmfd_maxpool_nhwc")
    return out, Ho, Wo


def global_avgpool(x, N, HW, C):
    out = torch.empty((N, C), device=x.device, dtype=torch.float32)
    _check(lib().mmfd_global_avgpool(dtype_code(x.dtype), N, HW, C, _ptr(x), _ptr(out), _stream()),
           "mmfd_global_avgpool")
    return out


def embed_bwd(ids, tts, dsum, dword, dpos, dtype_emb, padding_idx=-1):
    """deterministic embedding-table gradients (csrc/embed_bwd.hip): sort-by-id word scatter-add"""
    B, L = ids.shape
    D = dsum.shape[-1]
    nws = lib().mmfd_embed_bwd_workspace_bytes(B, L, D)
    if nws < 0:
        raise RuntimeError("mmfd_embed_bwd_workspace_bytes failed")
    ws = torch.empty(max(nws, 1), device=dsum.device, dtype=torch.uint8)
    vocab = dword.shape[0] if dword is not None else 0  # the sort covers the id bits of the vocabulary only
    _check(lib().mmfd_embed_bwd(dtype_code(dsum.dtype), B, L, D, vocab, _ptr(ids), _ptr(tts) if tts is not None else None,
                                _ptr(dsum), _ptr(dword), _ptr(dpos), _ptr(dtype_emb), int(padding_idx), _ptr(ws), nws,
                                _stream()),
           "mmfd_embed_bwd")


def patchify(pixels, P, dtype):
    B, C, Hh, Ww = pixels.shape
    npch = (Hh // P) * (Ww // P)
    out = torch.empty((B * npch, C * P * P), device=pixels.device, dtype=dtype)
    _check(lib().mmfd_patchify(dtype_code(dtype), B, C, Hh, Ww, P, _ptr(pixels.contiguous().float()), _ptr(out),
                               _stream()), "mmfd_patchify")
    return out


def vit_tokens_fwd(patch, B, cls, pos):
    NP = patch.shape[0] // B
    D = patch.shape[1]
    out = torch.empty((B, NP + 1, D), device=patch.device, dtype=patch.dtype)
    _check(lib().mmfd_vit_tokens_fwd(dtype_code(patch.dtype), B, NP, D, _ptr(patch), _ptr(cls), _ptr(pos), _ptr(out),
                                     _stream()), "mmfd_vit_tokens_fwd")
    return out


def vit_tokens_bwd(dout, want_dpatch=True):
    B, T, D = dout.shape
    NP = T - 1
    dpatch = torch.empty((B * NP, D), device=dout.device, dtype=dout.dtype) if want_dpatch else None
    dcls = torch.empty(D, device=dout.device, dtype=torch.float32)
    dpos = torch.empty((T, D), device=dout.device, dtype=torch.float32)
    _check(lib().mmfd_vit_tokens_bwd(dtype_code(dout.dtype), B, NP, D, _ptr(dout.contiguous()), _ptr(dpatch),
                                     _ptr(dcls), _ptr(dpos), None, 0, _stream()), "mmfd_vit_tokens_bwd")
    return dpatch, dcls, dpos


def adamw(table_dev, n, max_numel, lr, beta1, beta2, eps, weight_decay):
    _ops().adamw(table_dev, int(n), int(max_numel), float(lr), float(beta1), float(beta2), float(eps),
                 float(weight_decay))


def dropout_hash(seed: int, salt: int, index: int) -> int:
    return int(lib().mmfd_dropout_hash(seed & 0xFFFFFFFFFFFFFFFF, salt & 0xFFFFFFFFFFFFFFFF, index))


# ------------------------------------------------------------------------------------------------
# retrieval scoring (csrc/retrieval.hip)
# ------------------------------------------------------------------------------------------------
_CORPUS_CODES = {torch.float32: F32, torch.bfloat16: BF16, torch.float16: F16}


def cosine_scores(queries, corpus, mode=COS_PAIR, eps=1e-6, out=None):
    """fp32 [Q, N] cosine scores of fp32 queries [Q, D] against a corpus [N, D] (fp32 / bf16 / fp16)."""
    _require_cuda(queries, corpus, out)
    if queries.dim() == 1:
        queries = queries.unsqueeze(0)
    queries = queries.float().contiguous()
    corpus = corpus.contiguous()
    Q, D = queries.shape
    N = corpus.shape[0]
    if corpus.shape[1] != D:
        raise ValueError(f"query dim {D} != corpus dim {corpus.shape[1]}")
    if corpus.dtype not in _CORPUS_CODES:
        raise TypeError(f"unsupported corpus dtype {corpus.dtype}")
    if out is None:
        out = torch.empty(Q, N, device=corpus.device, dtype=torch.float32)
    _ld(corpus)
    _ops().cosine_scores(queries, corpus, int(mode), float(eps), out)
    return out


def topk(scores, k):
    """Per row of fp32 scores [Q, N]: the k largest, descending, ties -> lower index first.
    Returns (values fp32 [Q, k], indices int64 [Q, k]); missing entries are -inf / -1."""
    _require_cuda(scores)
    Q, N = scores.shape
    val = torch.empty(Q, k, device=scores.device, dtype=torch.float32)
    idx = torch.empty(Q, k, device=scores.device, dtype=torch.int64)
    _ld(scores)
    _ops().topk(scores, int(k), val, idx)
    return val, idx


# -------------------------------------------------------------------------------------------------
# Swinv2 (csrc/swin.hip)
# -------------------------------------------------------------------------------------------------
def row_gather(src, idx, B, rows_out, G=1, out=None):
    """src [B*src_rows, C] -> out [B*rows_out, G*C] with out row (b, r) = concat_g src row
    (b, idx[r*G+g]); idx int32 [rows_out*G] (one image's table, shared by the batch)"""
    _require_cuda(src, idx)
    if idx.dtype != torch.int32 or idx.numel() != rows_out * G:
        raise ValueError("row_gather: idx must be int32 [rows_out*G]")
    if not src.is_contiguous() or src.shape[0] % B:
        raise ValueError("row_gather: src must be contiguous [B*src_rows, C]")
    C = src.shape[1]
    if out is None:
        out = torch.empty((B * rows_out, G * C), device=src.device, dtype=src.dtype)
    _check(lib().mmfd_row_gather(B, rows_out, G, C * src.element_size(), src.shape[0] // B, _ptr(src), _ptr(idx),
                                 _ptr(out), _stream()), "mmfd_row_gather")
    return out


def swin_cpb(coords, w1, b1, w2, out=None):
    """continuous position-bias MLP table [T, H] (fp32) from coords [T, 2], w1 [512, 2], b1 [512], w2 [H, 512]"""
    _require_cuda(coords, w1, b1, w2)
    T, H = coords.shape[0], w2.shape[0]
    if w1.shape != (512, 2) or w2.shape[1] != 512:
        raise ValueError("swin_cpb: the position-bias MLP has 512 hidden units")
    ts = [t.float().contiguous() for t in (coords, w1, b1, w2)]
    if out is None:
        out = torch.empty((T, H), device=coords.device, dtype=torch.float32)
    _check(lib().mmfd_swin_cpb(T, H, *[_ptr(t) for t in ts], _ptr(out), _stream()), "mmfd_swin_cpb")
    return out


def swin_bias(table, rpi, L, mask=None, out=None):
    """[nW, H, L, L] fp32 = 16 sigmoid(table[rpi]) (+ 2 * mask[nW, L, L]); nW = 1 without a mask"""
    _require_cuda(table, rpi)
    H = table.shape[1]
    nW = mask.shape[0] if mask is not None else 1
    if out is None:
        out = torch.empty((nW, H, L, L), device=table.device, dtype=torch.float32)
    _check(lib().mmfd_swin_bias(nW, H, L, _ptr(table), _ptr(rpi), _ptr(mask) if mask is not None else None,
                                _ptr(out), _stream()), "mmfd_swin_bias")
    return out


def swin_qk_norm(qkv, H, d, logit_scale, max_log):
    """in place on packed QKV rows [rows, >= 2*H*d]: cosine-attention q (times the head's clamped
    exp(logit_scale)) and k"""
    _require_cuda(qkv, logit_scale)
    ls = logit_scale.float().contiguous()
    _check(lib().mmfd_swin_qk_norm(dtype_code(qkv.dtype), qkv.shape[0], H, d, _ptr(qkv), _ld(qkv), _ptr(ls),
                                   float(max_log), _stream()), "mmfd_swin_qk_norm")
    return qkv
