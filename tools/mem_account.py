"""Device-memory accounting of the bs=256 full fine-tune step, run on the GPU box:

  python tools/mem_account.py [--precision fp32] [--batch 256] [--out profiles/r04_memory.json]

Separately measured, in GiB:
  resident        parameters + gradients + AdamW moments (+ bf16 shadows) between steps
  saved_fwd       what the forward keeps for the backward (memory_allocated after forward + loss
                  minus before), and of it the split-operand planes still alive at that point
                  (activation planes saved for the weight-gradient GEMMs; the per-call weight
                  planes are counted apart)
  eager_peak      max_memory_allocated over one eager step (forward, backward, AdamW)
  graph_pool      memory_reserved growth across FusionTrainer.capture() (the HIP graph's private
                  pool; the capture's own eager warm-up steps run first and use the normal pool)
  capture_peak    max_memory_allocated from before the capture to after the first replays (what
                  bench.py's peak_memory_gb reported through round 3)
"""
import argparse
import json
import os
import sys
import weakref

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

GiB = float(2 ** 30)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--precision", default="fp32")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from mmfd import blocks as Bk
    from mmfd import kernels as K
    from mmfd.dataset import synthetic_batch
    from mmfd.train import build_flagship

    dev = torch.device("cuda", 0)
    tr = build_flagship(dev, a.precision, seed=42)
    batch = synthetic_batch(a.batch, seed=1000, device=dev)
    tr.step(batch)  # optimizer state, shadows
    torch.cuda.synchronize()
    out = {"precision": a.precision, "batch_pairs": a.batch}

    # planes made during a forward: activation planes (split3 of GEMM inputs, producer-written
    # planes) vs the per-call weight planes (StepCtx.wplanes)
    live = {"act": [], "w": []}
    split3, wplanes, out_planes, new_planes = K.split3, Bk.StepCtx.wplanes, Bk.out_planes, Bk.new_planes
    in_w = [False]

    def split3_w(x, out=None):
        r = split3(x, out)
        live["w" if in_w[0] else "act"].append(weakref.ref(r))
        return r

    def wplanes_w(self, W):
        in_w[0] = True
        try:
            return wplanes(self, W)
        finally:
            in_w[0] = False

    def out_planes_w(*args, **kw):
        r = out_planes(*args, **kw)
        if r[0] is not None:
            live["act"].append(weakref.ref(r[0]))
        return r

    def new_planes_w(*args, **kw):
        r = new_planes(*args, **kw)
        if r is not None:
            live["act"].append(weakref.ref(r))
        return r

    K.split3, Bk.StepCtx.wplanes, Bk.out_planes, Bk.new_planes = split3_w, wplanes_w, out_planes_w, new_planes_w
    try:
        tr.optimizer.zero_grad(set_to_none=True)
        torch.cuda.synchronize()
        m0 = torch.cuda.memory_allocated(dev)
        outs = tr._head_forward(batch)
        loss = tr.loss(outs, batch["labels"].to(dev))
        torch.cuda.synchronize()
        m1 = torch.cuda.memory_allocated(dev)

        def alive(kind):
            seen, n = set(), 0
            for r in live[kind]:
                t = r()
                if t is not None and t.data_ptr() not in seen:
                    seen.add(t.data_ptr())
                    n += t.numel() * t.element_size()
            return n
        out["resident_gib"] = round(m0 / GiB, 2)
        out["saved_fwd_gib"] = round((m1 - m0) / GiB, 2)
        out["saved_act_planes_gib"] = round(alive("act") / GiB, 2)
        out["saved_weight_planes_gib"] = round(alive("w") / GiB, 2)
        g = torch.tensor([1.0] + [0.0] * (loss.numel() - 1), device=dev)
        torch.autograd.backward(loss, g)
        tr.optimizer.step()
        del outs, loss
    finally:
        K.split3, Bk.StepCtx.wplanes, Bk.out_planes, Bk.new_planes = split3, wplanes, out_planes, new_planes
    torch.cuda.synchronize()
    torch.cuda.reset_peak_memory_stats(dev)
    base = torch.cuda.memory_allocated(dev)
    tr.step(batch)
    torch.cuda.synchronize()
    out["eager_peak_gib"] = round(torch.cuda.max_memory_allocated(dev) / GiB, 2)
    out["eager_step_transient_gib"] = round((torch.cuda.max_memory_allocated(dev) - base) / GiB, 2)
    out["params_m"] = round(sum(p.numel() for p in tr.params) / 1e6, 2)
    torch.cuda.empty_cache()
    r0 = torch.cuda.memory_reserved(dev)
    torch.cuda.reset_peak_memory_stats(dev)
    tr.capture(batch, warmup=1)
    tr.replay()
    tr.replay()
    torch.cuda.synchronize()
    out["graph_pool_gib"] = round((torch.cuda.memory_reserved(dev) - r0) / GiB, 2)
    out["capture_peak_gib"] = round(torch.cuda.max_memory_allocated(dev) / GiB, 2)
    out["reserved_after_capture_gib"] = round(torch.cuda.memory_reserved(dev) / GiB, 2)
    print(json.dumps(out), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
