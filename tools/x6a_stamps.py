"""Diagnostic: phase cycle counts of the split-operand fp32 attention forward (attn_fwd_x6_kernel)
from s_memtime stamps (a separate -DMMFD_X6A_STAMPS build of libmmfd_hip under tools/_stamps/; the
product library is untouched). Per wave: 0 entry, 1 K/V planes staged (after the barrier), 2 first
query block's Q fragments split, 3.. after each full 64-key chunk, 7 after the last chunk, 8 after
the block's stores, 9 exit.
  python tools/x6a_stamps.py [build | bert | vit]"""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SRC = os.path.join(ROOT, "multimodal-misinformation-detection_amd", "csrc")
LIB = os.path.join(ROOT, "tools", "_stamps", "libmmfd_hip_x6astamps.so")

if len(sys.argv) > 1 and sys.argv[1] == "build":
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    o = os.path.join(os.path.dirname(LIB), "attention.x6a.o")
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-fPIC", "-std=c++17", "--offload-arch=gfx950", "-mllvm",
                    "-amdgpu-mfma-vgpr-form", "-DMMFD_X6A_STAMPS", "-c", os.path.join(SRC, "attention.hip"), "-o", o],
                   check=True)
    objs = [os.path.join(SRC, "build", f) for f in sorted(os.listdir(os.path.join(SRC, "build")))
            if f.endswith(".o") and f not in ("attention.o", "torch_ops.o")]
    subprocess.run(["/opt/rocm/bin/hipcc", "-shared", "-fPIC", "--offload-arch=gfx950", "-o", LIB, o] + objs, check=True)
    sys.exit(0)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import mmfd  # noqa: E402,F401
from mmfd import kernels as K  # noqa: E402

K.load(LIB)
lib = K.lib()
lib.mmfd_debug_x6a_stamps.restype = ctypes.c_int
lib.mmfd_debug_x6a_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int64]
which = sys.argv[1] if len(sys.argv) > 1 else "vit"
L, masked, p = (197, False, 0.0) if which == "vit" else (128, True, 0.1)
B, H, D = 512, 12, 64
dev = "cuda"
g = torch.Generator(device="cpu").manual_seed(0)
qkv = torch.randn(B, L, 3 * H * D, generator=g).to(dev)
q, k, v = qkv[..., :H * D], qkv[..., H * D:2 * H * D], qkv[..., 2 * H * D:]
kb = None
if masked:
    mask = torch.ones(B, L, dtype=torch.long)
    mask[::2, L * 3 // 4:] = 0
    kb = K.mask_to_bias(mask.to(dev))
kw = dict(key_bias=kb, dropout_p=p, seed=K.Seed(5), salt=K.salt_of("bench")) if p > 0 else dict(key_bias=kb)
for _ in range(3):
    o, lse = K.attn_fwd(q, k, v, H, **kw)
torch.cuda.synchronize()
nwg = min(8192, B * H)
buf = np.zeros(8192 * 8 * 16, dtype=np.uint64)
assert lib.mmfd_debug_x6a_stamps(buf.ctypes.data, buf.nbytes) == 0
st = buf.reshape(8192, 8, 16)[:nwg].astype(np.int64)
t0 = st[:, :, 0].min(axis=1, keepdims=True)
rel = st - t0[:, :, None]
names = {1: "staged", 2: "Q split", 3: "chunk0", 4: "chunk1", 5: "chunk2", 7: "last chunk", 8: "stores", 9: "exit"}
prev = 0
print(f"{which}: per-wave cycles from the workgroup's first entry (mean over {nwg} workgroups)")
for w in range(8):
    row = []
    for s in (1, 2, 3, 4, 5, 7, 8, 9):
        vals = rel[:, w, s]
        ok = st[:, w, s] > 0
        if ok.sum() == 0:
            continue
        row.append(f"{names[s]} {vals[ok].mean():8.0f}")
    print(f"  wave {w}: " + " | ".join(row))
wg = (st[:, :, 9].max(axis=1) - st[:, :, 0].min(axis=1))
print(f"  workgroup lifetime: mean {wg.mean():.0f} cycles; launch span {(st[:, :, 9].max() - st[:, :, 0].min()):.0f}")
