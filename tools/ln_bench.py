"""LayerNorm forward / backward at the encoder shapes (BERT 65,536 and ViT 100,864 token rows of
768, the fusion head's rows of 256), bf16 and fp32: microseconds per call and the algorithmic HBM
rate (forward x in, y out; backward dy, x, dx_add in, dx and dx_drop out — the post-LN BERT
layer's form). python tools/ln_bench.py [--iters N]"""
import argparse
import sys, os

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from mmfd import kernels as K  # noqa: E402


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    seed = K.Seed(5, device="cuda")
    for dt in (torch.bfloat16, torch.float32):
        for R, W in ((65536, 768), (100864, 768), (16384, 256)):
            x = torch.randn(R, W, device="cuda").to(dt)
            dy = torch.randn(R, W, device="cuda").to(dt)
            add = torch.randn(R, W, device="cuda").to(dt)
            g = torch.randn(W, device="cuda")
            b = torch.randn(W, device="cuda")
            y, mean, rstd = K.layernorm_fwd(x, g, b, 1e-12)
            dx, dd = torch.empty_like(x), torch.empty_like(x)
            dg, db = torch.empty(W, device="cuda"), torch.empty(W, device="cuda")
            tf = timed(lambda: K.layernorm_fwd(x, g, b, 1e-12, out=y), a.iters)
            tb = timed(lambda: K.layernorm_bwd(dy, x, g, mean, rstd, dx=dx, dx_add=add, dgamma=dg, dbeta=db,
                                               dx_drop=dd, dropout_p=0.1, seed=seed, salt=3), a.iters)
            eb = x.element_size() * R * W
            print(f"RESULT {str(dt)[6:]:8s} {R:6d}x{W:4d} fwd {tf:8.1f} us {2 * eb / tf / 1e3:6.2f} GB/s   "
                  f"bwd {tb:8.1f} us {5 * eb / tb / 1e3:6.2f} GB/s", flush=True)


if __name__ == "__main__":
    main()
