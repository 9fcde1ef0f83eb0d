"""Diagnostic: where the four-wave split-operand GEMM (gemm256_x6w_kernel) spends a K-step and a tile,
from s_memtime stamps (a separate -DMMFD_W4_STAMPS build of libmmfd_hip under tools/_stamps/; the
product library is untouched). Stamps of one mid-loop K-step: 0 loop top, 1 own DMA landed
(vmcnt(0)), 2 past barrier 1, 3 subtile 0's MFMAs issued, 4 subtile 1's issued + lgkmcnt(0),
5 past barrier 2, 6 the step's last MFMAs issued; per tile: 16 start, 17 loop end, 18 row sums
done, 19 epilogue stores retired.
  python tools/w4_stamps.py build [variant DEFINE=VAL ...]     (in the build container)
  W4_VARIANT=<variant> python tools/w4_stamps.py [M N K [fwd|dx|dw]]   (on the GPU box)"""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SRC = os.path.join(ROOT, "multimodal-misinformation-detection_amd", "csrc")
LIB = os.path.join(ROOT, "tools", "_stamps", "libmmfd_hip_w4stamps.so")


def build(variant="", defines=()):
    out = LIB.replace(".so", f"{variant}.so")
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    objs = []
    for f in sorted(os.listdir(SRC)):
        if not f.endswith(".hip"):
            continue
        w4 = f == "gemm_x6w.hip"
        o = os.path.join(os.path.dirname(LIB), f + (f".w4{variant}.o" if w4 else ".w4.o"))
        if w4 or not os.path.exists(o):
            flags = ["-fno-slp-vectorize", *[f"-D{d}" for d in defines]] if w4 else ["-mllvm", "-amdgpu-mfma-vgpr-form"]
            if f == "gemm_x6f.hip":
                flags.append("-fno-slp-vectorize")
            subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-fPIC", "-std=c++17", "--offload-arch=gfx950",
                            "-DMMFD_W4_STAMPS", *flags, "-c", os.path.join(SRC, f), "-o", o], check=True)
        objs.append(o)
    subprocess.run(["/opt/rocm/bin/hipcc", "-shared", "-fPIC", "--offload-arch=gfx950", "-o", out] + objs, check=True)


if len(sys.argv) > 1 and sys.argv[1] == "build":
    build(sys.argv[2] if len(sys.argv) > 2 else "", sys.argv[3:])
    sys.exit(0)
VARIANT = os.environ.get("W4_VARIANT", "")
LIB = LIB.replace(".so", f"{VARIANT}.so")
os.environ["MMFD_X6W"] = "1"

import numpy as np  # noqa: E402
import torch  # noqa: E402

import mmfd  # noqa: E402,F401
from mmfd import kernels as K  # noqa: E402

K.load(LIB)
lib = K.lib()
lib.mmfd_debug_w4_stamps.restype = ctypes.c_int
lib.mmfd_debug_w4_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int64]
lib.mmfd_debug_set_x6w.argtypes = [ctypes.c_int]
lib.mmfd_debug_set_x6w(1)
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
epi = os.environ.get("W4_EPI", "plain")
if epi == "gelu":
    kw.update(bias=torch.randn(N, device=dev), act=K.ACT_GELU, aux=torch.empty(M, N, device=dev),
              out_planes=torch.empty(3, M, N, device=dev, dtype=torch.bfloat16), write_out=False)
for _ in range(3):
    K.gemm(A, B, out=out, a_planes=ap, b_planes=bp, **kw)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(5):
    K.gemm(A, B, out=out, a_planes=ap, b_planes=bp, **kw)
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) * 1000 / 5
nblk = min(((M + 255) // 256) * ((N + 255) // 256), 4096)
buf = np.zeros(4096 * 4 * 24, np.uint64)
assert lib.mmfd_debug_w4_stamps(buf.ctypes.data, buf.nbytes) == 0
st = buf.reshape(4096, 4, 24)[:nblk].astype(np.int64)
print(f"variant '{VARIANT}' M={M} N={N} K={Kd} {lay} epilogue {epi}: {us:.1f} us/launch "
      f"({2 * M * N * Kd / us / 1e6:.1f} TF); {nblk} blocks; cycles median / p90 over blocks x waves")


def q(x):
    x = x.reshape(-1)
    return f"{np.median(x):8.0f} / {np.percentile(x, 90):8.0f}"


names = ["vmcnt(0) wait", "barrier 1", "B+A0 reads -> subtile 0 issued", "subtile 1 + lgkmcnt(0)", "barrier 2",
         "subtiles 2-7"]
for k in range(6):
    print(f"  step {names[k]:34s} {q(st[:, :, k + 1] - st[:, :, k])}")
print(f"  step total                         {q(st[:, :, 6] - st[:, :, 0])}")
print(f"  tile main loop                     {q(st[:, :, 17] - st[:, :, 16])}")
print(f"  tile row sums                      {q(st[:, :, 18] - st[:, :, 17])}")
print(f"  tile epilogue (stores retired)     {q(st[:, :, 19] - st[:, :, 18])}")
