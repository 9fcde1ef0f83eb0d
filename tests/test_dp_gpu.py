"""Data-parallel training step on the HIP path: 2 ranks (gloo, both on cuda:0 — the box has one
GPU) each run FusionTrainer.step on half of a batch with the overlapped gradient all-reduce; the
ranks build their replicas from DIFFERENT seeds and FusionTrainer broadcasts rank 0's weights.
The averaged gradients must equal the single-process gradients of the full batch (fp32, dropout
off; the loss is a batch mean, so mean-of-halves == full-batch gradient up to fp32 rounding), and
after a second step both replicas hold bitwise-identical parameters.
Tolerance: 2e-4 relative to each tensor's max |grad| (the floor of tests/smoke_impl.compare_step).
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _grads(tr):
    out = {}
    for pre, m in (("bert.", tr.text_encoder), ("vit.", tr.image_encoder), ("head.", tr.head)):
        for k, p in m.named_parameters():
            out[pre + k] = p.grad.detach().float().cpu().numpy().copy() if p.grad is not None else None
    return out


def _half(batch, rank, world):
    B = batch["labels"].shape[0]
    h = B // world
    sl = slice(rank * h, (rank + 1) * h)
    return {"input_ids": torch.cat([batch["input_ids"][:B][sl], batch["input_ids"][B:][sl]]),
            "attention_mask": torch.cat([batch["attention_mask"][:B][sl], batch["attention_mask"][B:][sl]]),
            "pixel_values": torch.cat([batch["pixel_values"][:B][sl], batch["pixel_values"][B:][sl]]),
            "labels": batch["labels"][sl]}


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mmfd.dp import GradAllReduce
        from mmfd.train import FusionTrainer
        from tests.smoke_impl import build_pair, tiny_batch
        # each rank initialises from its OWN seed: FusionTrainer broadcasts rank 0's weights
        t0, _ = build_pair("fp32", dropout=0.0, seed=5 + 11 * rank)
        dp = GradAllReduce(bucket_mb=0.05)  # many buckets -> several in flight during backward
        tr = FusionTrainer(t0.text_encoder, t0.image_encoder, t0.head, lr=1e-3, precision="fp32", dp=dp)
        b = _half(tiny_batch(4, seed=21), rank, world)
        tr.step({k: v.cuda() for k, v in b.items()})
        torch.cuda.synchronize()
        g1 = _grads(tr)
        tr.step({k: v.cuda() for k, v in _half(tiny_batch(4, seed=22), rank, world).items()})
        torch.cuda.synchronize()
        params = {k: v.detach().cpu().numpy().copy() for m, pre in ((tr.text_encoder, "bert."), (tr.image_encoder, "vit."),
                                                                      (tr.head, "head.")) for k, v in
                  ((pre + n, p) for n, p in m.named_parameters())}
        q.put((rank, g1, params))
    finally:
        dist.destroy_process_group()


def test_dp_two_ranks_match_full_batch():
    from tests.smoke_impl import build_pair, tiny_batch
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res, params = {}, {}
    for _ in range(world):
        r, g1, pr = q.get(timeout=300)
        res[r], params[r] = g1, pr
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for k in params[0]:  # replicas started from different seeds, trained 2 steps: identical
        assert (params[0][k] == params[1][k]).all(), k
    tr, _ = build_pair("fp32", dropout=0.0)
    tr.step({k: v.cuda() for k, v in tiny_batch(4, seed=21).items()})
    torch.cuda.synchronize()
    full = _grads(tr)
    floor = 1e-3 * max(abs(g).max() for g in full.values() if g is not None)
    for k, g in full.items():
        if g is None:
            continue
        scale = max(abs(g).max(), floor)
        for r in range(world):
            e = abs(res[r][k] - g).max() / scale
            assert e < 2e-4, f"rank {r} {k}: {e:.2e}"
