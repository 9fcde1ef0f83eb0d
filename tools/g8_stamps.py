"""Diagnostic: per-wave phase times of the 256x256 GEMM from s_memtime stamps (a separate
-DMMFD_G8_STAMPS build of libmmfd_hip under tools/_stamps/; the product library is untouched).
Stamps: 0 start, 1 mainloop done, 2 after the re-align + vmcnt(0) + barrier, 3 staging written,
4 after the staging barrier, 5 first 128 rows read back + stored, 6 epilogue issued, 7 stores
retired (vmcnt(0)); bf16 main-loop segments of K-tile 4 (stamps 8-16): X reads + refill issue +
vmcnt, X pre-barrier, X MFMAs, X barrier, then the same for Y.
Stamps 17-20 split each read side into fragment reads / refill issue / vmcnt wait.
python tools/g8_stamps.py [M N K [plain|gelu|gelubwd] [bf16|fp32]]"""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

SRC = os.path.join(ROOT, "multimodal-misinformation-detection_amd", "csrc")
LIB = os.path.join(ROOT, "tools", "_stamps", "libmmfd_hip_stamps.so")
if not os.path.exists(LIB):
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    objs = []
    for f in sorted(os.listdir(SRC)):
        if f.endswith(".hip"):
            o = os.path.join(os.path.dirname(LIB), f + ".o")
            extra = ["-fno-slp-vectorize"] if f == "gemm_x6f.hip" else []  # the product build's flags
            subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-fPIC", "-std=c++17", "--offload-arch=gfx950", "-mllvm",
                            "-amdgpu-mfma-vgpr-form", *extra, "-DMMFD_G8_STAMPS", "-c", os.path.join(SRC, f), "-o", o],
                           check=True)
            objs.append(o)
    subprocess.run(["/opt/rocm/bin/hipcc", "-shared", "-fPIC", "--offload-arch=gfx950", "-o", LIB] + objs, check=True)

import mmfd  # noqa: E402,F401
from mmfd import kernels as K  # noqa: E402

K.load(LIB)
lib = K.lib()
lib.mmfd_debug_g8_stamps.restype = ctypes.c_int
lib.mmfd_debug_g8_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int64]
M, N, Kd = (int(x) for x in sys.argv[1:4]) if len(sys.argv) > 3 else (65536, 3072, 768)
kind = sys.argv[4] if len(sys.argv) > 4 else "plain"
dt = torch.float32 if (len(sys.argv) > 5 and sys.argv[5] == "fp32") else torch.bfloat16
A = torch.randn(M, Kd, device="cuda").to(dt)
B = torch.randn(N, Kd, device="cuda").to(dt)
out = torch.empty(M, N, device="cuda", dtype=dt)
aux = torch.randn(M, N, device="cuda").to(dt)
bias = torch.randn(N, device="cuda")
for _ in range(5):
    if kind == "gelu":
        K.gemm(A, B, out=out, bias=bias, act=K.ACT_GELU, aux=aux)
    elif kind == "gelubwd":
        K.gemm(A, B, out=out, act=K.ACT_GELU_BWD, aux=aux)
    else:
        K.gemm(A, B, out=out)
torch.cuda.synchronize()
nblk = min((M // 256) * (N // 256), 16384)
NS = 24
buf = np.zeros(16384 * 8 * NS, np.uint64)
assert lib.mmfd_debug_g8_stamps(buf.ctypes.data, buf.nbytes) == 0
full = buf.reshape(16384, 8, NS)[:nblk].astype(np.int64)
st = full[:, :, :8]
d = np.diff(st, axis=2)  # [blocks, waves, 7]
names = ["mainloop", "realign+vmcnt+barrier", "stage writes", "stage barrier", "rows 0-127 epilogue",
         "rows 128-255 epilogue", "store drain"]
print(f"M={M} N={N} K={Kd} {kind}: {nblk} blocks; cycles per phase (median / p90 over waves)")
for i, n in enumerate(names):
    v = d[:, :, i].ravel()
    print(f"  {n:24s} {np.median(v):9.0f} {np.percentile(v, 90):9.0f}")
tot = st[:, :, 7] - st[:, :, 0]
print(f"  {'total':24s} {np.median(tot):9.0f} {np.percentile(tot, 90):9.0f}")
if dt == torch.bfloat16 and Kd >= 5 * 64:
    seg = np.diff(full[:, :, 8:17], axis=2)
    sn = ["X reads+issue+wait", "X pre-barrier", "X MFMAs", "X barrier", "Y reads+issue+wait", "Y pre-barrier",
          "Y MFMAs", "Y barrier"]
    print("K-tile 4 segments (median / p90 over waves):")
    for i, n in enumerate(sn):
        v = seg[:, :, i].ravel()
        print(f"  {n:24s} {np.median(v):9.0f} {np.percentile(v, 90):9.0f}")
    if True:  # the reads / issue / wait split
        for n, a, b in (("X reads", 8, 17), ("X refill issue", 17, 18), ("X vmcnt wait", 18, 9),
                        ("Y reads", 12, 19), ("Y refill issue", 19, 20), ("Y vmcnt wait", 20, 13)):
            v = (full[:, :, b] - full[:, :, a]).ravel()
            print(f"  {n:24s} {np.median(v):9.0f} {np.percentile(v, 90):9.0f}")
    kt = full[:, :, 16] - full[:, :, 8]
    print(f"  {'K-tile':24s} {np.median(kt):9.0f} {np.percentile(kt, 90):9.0f}")
