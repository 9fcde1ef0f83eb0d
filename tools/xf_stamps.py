"""Diagnostic: per-phase cycle counts of the fused-plane split-operand GEMM (gemm256_x6f_kernel) from
s_memtime stamps of one mid-loop K-step (a separate -DMMFD_XF_STAMPS build of libmmfd_hip under
tools/_stamps/; the product library is untouched). Per phase p: stamp 4p = read phase start (after
the barrier), 4p+1 = reads + DMA issued + vmcnt wait done, 4p+2 = after the pre-MFMA barrier,
4p+3 = the phase's 48 MFMAs and adds issued.
  python tools/xf_stamps.py [build | M N K [fwd|dx|dw]]"""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SRC = os.path.join(ROOT, "multimodal-misinformation-detection_amd", "csrc")
LIB = os.path.join(ROOT, "tools", "_stamps", "libmmfd_hip_xfstamps.so")


def build(variant="", defines=()):
    """the stamps library (all kernels; gemm_x6f.hip with -DMMFD_XF_STAMPS and `defines`); the
    other translation units' objects are reused between variants"""
    out = LIB.replace(".so", f"{variant}.so")
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    objs = []
    for f in sorted(os.listdir(SRC)):
        if not f.endswith(".hip"):
            continue
        xf = f == "gemm_x6f.hip"
        o = os.path.join(os.path.dirname(LIB), f + (f".xf{variant}.o" if xf else ".xf.o"))
        if xf or not os.path.exists(o):
            extra = ["-fno-slp-vectorize", *[f"-D{d}" for d in defines]] if xf else []
            subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-fPIC", "-std=c++17", "--offload-arch=gfx950", "-mllvm",
                            "-amdgpu-mfma-vgpr-form", "-DMMFD_XF_STAMPS", *extra, "-c", os.path.join(SRC, f), "-o", o],
                           check=True)
        objs.append(o)
    subprocess.run(["/opt/rocm/bin/hipcc", "-shared", "-fPIC", "--offload-arch=gfx950", "-o", out] + objs, check=True)


if len(sys.argv) > 1 and sys.argv[1] == "build":  # build [variant DEFINE=VAL ...]
    build(sys.argv[2] if len(sys.argv) > 2 else "", sys.argv[3:])
    sys.exit(0)
VARIANT = os.environ.get("XF_VARIANT", "")
LIB = LIB.replace(".so", f"{VARIANT}.so")

import numpy as np  # noqa: E402
import torch  # noqa: E402

import mmfd  # noqa: E402,F401
from mmfd import kernels as K  # noqa: E402

K.load(LIB)
lib = K.lib()
lib.mmfd_debug_xf_stamps.restype = ctypes.c_int
lib.mmfd_debug_xf_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int64]
M, N, Kd = (int(x) for x in sys.argv[1:4]) if len(sys.argv) > 3 else (65536, 3072, 768)
lay = sys.argv[4] if len(sys.argv) > 4 else "fwd"
dev = "cuda"
if lay == "fwd":
    A = torch.randn(M, Kd, device=dev); B = torch.randn(N, Kd, device=dev); kw = {}
elif lay == "dx":
    A = torch.randn(M, Kd, device=dev); B = torch.randn(Kd, N, device=dev); kw = dict(trans_b=True)
else:
    A = torch.randn(Kd, M, device=dev); B = torch.randn(Kd, N, device=dev); kw = dict(trans_a=True, trans_b=True)
ap, bp = K.split3(A), K.split3(B)
out = torch.empty(M, N, device=dev)
epi = os.environ.get("XF_EPI", "plain")  # plain | gelu (bias + GELU + saved pre-activation, output as planes only)
if epi == "gelu":
    kw.update(bias=torch.randn(N, device=dev), act=K.ACT_GELU, aux=torch.empty(M, N, device=dev),
              out_planes=torch.empty(3, M, N, device=dev, dtype=torch.bfloat16), write_out=False)
for _ in range(5):
    K.gemm(A, B, out=out, a_planes=ap, b_planes=bp, **kw)
torch.cuda.synchronize()
nblk = min(((M + 255) // 256) * ((N + 255) // 256), 4096)
buf = np.zeros(4096 * 8 * 20, np.uint64)
assert lib.mmfd_debug_xf_stamps(buf.ctypes.data, buf.nbytes) == 0
st = buf.reshape(4096, 8, 20)[:nblk].astype(np.int64)
print(f"M={M} N={N} K={Kd} {lay} epilogue {epi}: {nblk} blocks; cycles (median / p90 over blocks), row 0 = waves 0-3, row 1 = 4-7")
for row, ws in (("row0", slice(0, 4)), ("row1", slice(4, 8))):
    s = st[:, ws, :]
    for p in range(4):
        r = s[:, :, 4 * p + 1] - s[:, :, 4 * p]
        b = s[:, :, 4 * p + 2] - s[:, :, 4 * p + 1]
        c = s[:, :, 4 * p + 3] - s[:, :, 4 * p + 2]
        nxt = (s[:, :, 4 * p + 4] if p < 3 else None)
        line = (f"  {row} phase {p}: reads+dma+wait {np.median(r):6.0f}/{np.percentile(r, 90):6.0f}  "
                f"barrier {np.median(b):6.0f}/{np.percentile(b, 90):6.0f}  mfma issue {np.median(c):6.0f}/{np.percentile(c, 90):6.0f}")
        if nxt is not None:
            z = nxt - s[:, :, 4 * p + 3]
            line += f"  post-barrier {np.median(z):6.0f}/{np.percentile(z, 90):6.0f}"
        print(line)
    tot = s[:, :, 15] - s[:, :, 0]
    print(f"  {row} step (phase 0 start -> phase 3 mfma issued): {np.median(tot):.0f}/{np.percentile(tot, 90):.0f}"
          f"  (ideal: 4 x 768 MFMA cycles x 2 rows = 6144 per step per SIMD)")
    ml, ep = s[:, :, 17] - s[:, :, 16], s[:, :, 18] - s[:, :, 17]
    print(f"  {row} tile: main loop {np.median(ml):.0f}/{np.percentile(ml, 90):.0f}, epilogue (stores retired) "
          f"{np.median(ep):.0f}/{np.percentile(ep, 90):.0f} cycles")
