"""Attention kernels at the encoder shapes (bs=256 pairs -> 512 sequences x 12 heads, D=64):
BERT L=128 with key mask + dropout 0.1, ViT L=197 without. Prints per-kernel-call times.
BERT runs twice: the backward re-hashing the dropout mask, and reading the forward's keep-bitmask.
--ab-generic: every case also on the v2 kernels' generic mode 0 (mmfd_debug_set_attn_v2_generic)
python tools/attn_bench.py [--iters N] [--only bert|vit] [--fp32-mode split|native] [--planes] [--ab-generic]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import mmfd  # noqa: E402
from mmfd import kernels as K  # noqa: E402


def case(name, L, masked, p, iters, dtype=torch.bfloat16, planes=False, bitmask=False, B=512, H=12, D=64):
    dev = "cuda"
    g = torch.Generator(device="cpu").manual_seed(0)
    qkv = torch.randn(B, L, 3 * H * D, generator=g).to(dev, dtype)
    q, k, v = qkv[..., :H * D], qkv[..., H * D:2 * H * D], qkv[..., 2 * H * D:]
    dout = torch.randn(B, L, H * D, generator=g).to(dev, dtype)
    kb = None
    if masked:
        mask = torch.ones(B, L, dtype=torch.long)
        mask[::2, L * 3 // 4:] = 0
        kb = K.mask_to_bias(mask.to(dev))
    seed = K.Seed(5)
    kw = dict(key_bias=kb, dropout_p=p, seed=seed, salt=K.salt_of("bench")) if p > 0 else dict(key_bias=kb)
    if p > 0 and bitmask:  # the forward writes the keep-bitmask, the backward reads it
        kw["drop_mask"] = K.drop_mask_buffer(B, H, L, L, dev)
    o, lse = K.attn_fwd(q, k, v, H, **kw)
    dq = torch.empty_like(q); dk = torch.empty_like(k); dv = torch.empty_like(v)
    fkw, bkw = {}, {}
    if planes and dtype == torch.float32:
        # as the fp32 encoders run it: the output's planes from the forward, the packed dq|dk|dv
        # written as planes only by the backward
        fkw = dict(o_planes=torch.empty(3, B * L, H * D, device=dev, dtype=torch.bfloat16))
        dqkv = torch.empty(B, L, 3 * H * D, device=dev, dtype=dtype)
        dq, dk, dv = dqkv[..., :H * D], dqkv[..., H * D:2 * H * D], dqkv[..., 2 * H * D:]
        bkw = dict(dqkv_planes=torch.empty(3, B * L, 3 * H * D, device=dev, dtype=torch.bfloat16), planes_only=True)
    for _ in range(2):
        K.attn_fwd(q, k, v, H, out=o, **kw, **fkw)
        K.attn_bwd(q, k, v, o, lse, dout, H, dq=dq, dk=dk, dv=dv, **kw, **bkw)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    tf = tb = 0.0
    for _ in range(iters):
        ev[0].record()
        K.attn_fwd(q, k, v, H, out=o, **kw, **fkw)
        ev[1].record()
        K.attn_bwd(q, k, v, o, lse, dout, H, dq=dq, dk=dk, dv=dv, **kw, **bkw)
        ev[2].record()
        torch.cuda.synchronize()
        tf += ev[0].elapsed_time(ev[1])
        tb += ev[1].elapsed_time(ev[2])
    tf, tb = tf / iters, tb / iters
    fl = 4.0 * B * H * L * L * D
    print(f"{name}: fwd {tf * 1e3:7.1f} us ({fl / tf / 1e9:6.1f} TF/s)  bwd {tb * 1e3:7.1f} us "
          f"({2.5 * fl / tb / 1e9:6.1f} TF/s)", flush=True)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--only", default="")
    ap.add_argument("--dtype", default="bf16,fp32")
    ap.add_argument("--fp32-mode", default="split", help="fp32 attention: split (bf16 planes) or native")
    ap.add_argument("--planes", action="store_true", help="fp32: output / gradient planes as the encoders use them")
    ap.add_argument("--bert-p", type=float, default=0.1, help="BERT case dropout probability")
    ap.add_argument("--ab-generic", action="store_true")
    a = ap.parse_args()
    K.set_fp32_attn_mode(a.fp32_mode)
    import ctypes
    gen = K.lib().mmfd_debug_set_attn_v2_generic
    gen.argtypes, gen.restype = [ctypes.c_int], ctypes.c_int
    for dt, g in [(d, x) for d in a.dtype.split(",") for x in ((1, 0) if a.ab_generic else (0,))]:
        gen(g)
        if a.ab_generic:
            print(f"-- v2 {'generic mode 0' if g else 'fixed modes'}", flush=True)
        t = {"bf16": torch.bfloat16, "fp32": torch.float32}[dt]
        if a.only in ("", "bert"):
            case(f"{dt} bert L=128 mask p={a.bert_p} hash   ", 128, True, a.bert_p, a.iters, t, a.planes)
            if a.bert_p > 0:
                case(f"{dt} bert L=128 mask p={a.bert_p} bitmask", 128, True, a.bert_p, a.iters, t, a.planes, True)
        if a.only in ("", "vit"):
            case(f"{dt} vit  L=197          ", 197, False, 0.0, a.iters, t, a.planes)
        if a.only in ("", "head"):  # the fusion head: E = 256, 8 heads of D = 32, dropout, no key mask
            case(f"{dt} head L=128 D=32 p=0.1  ", 128, False, 0.1, a.iters, t, a.planes, B=256, H=8, D=32)
