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


# bounded worker waits (tests/mp_util.py)
from tests.mp_util import collect as _collect  # noqa: E402
from tests.mp_util import watchdog as _watchdog  # noqa: E402


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
    _watchdog()
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
    for r, g1, pr in _collect(procs, q, world):
        res[r], params[r] = g1, pr
    assert all(p.exitcode == 0 for p in procs)
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


# ---- full size: bert-base + ViT-B/16 + head, default 32 MB buckets, two encoder streams ----------
def _worker_full(rank, world, port, q):
    import torch.distributed as dist
    _watchdog()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mmfd.dp import GradAllReduce
        from mmfd.train import build_flagship
        from tests.smoke_impl import FULL, tiny_batch
        dp = GradAllReduce()  # the default 32 MB buckets, as bench.py / train.py use them
        assert dp.bucket_elems == 32 * (1 << 20) // 4
        # each rank from its OWN seed (rank 0's weights are broadcast), dropout off for the comparison
        tr = build_flagship("cuda", "fp32", dropout=0.0, dp=dp, seed=42 + 11 * rank, rank=rank, encoder_dropout=0.0)
        assert tr.concurrent  # text / image encoders on two HIP streams: buckets per stream
        b = _half(tiny_batch(2, cfg=FULL, seed=31), rank, world)
        tr.step({k: v.cuda() for k, v in b.items()})
        torch.cuda.synchronize()
        q.put((rank, _grads(tr), dict(dp.last_buckets)))
    except BaseException:
        import traceback
        q.put((rank, traceback.format_exc(), None))
        raise
    finally:
        dist.destroy_process_group()


def test_dp_full_size_default_buckets_two_streams():
    """config 4 at full size on the box's one GPU: 2 gloo ranks, bert-base + ViT-B/16 + the head at
    B = 1 pair per rank, the default 32 MB per-stream buckets over the 796 MB of fp32 gradients and
    both encoder streams; the averaged gradients equal the single-process B = 2 step's within 2e-4
    of each tensor's max (fp32, dropout off)."""
    from mmfd.train import build_flagship
    from tests.smoke_impl import FULL, tiny_batch
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker_full, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res, nb = {}, {}
    for r, g1, buckets in _collect(procs, q, world):
        assert buckets is not None, g1  # the worker's traceback
        res[r], nb[r] = g1, buckets
    assert all(p.exitcode == 0 for p in procs)
    print(f"buckets per stream: {nb[0]}", flush=True)
    assert len(nb[0]) == 2 and sum(nb[0].values()) >= 20, nb[0]  # buckets on both streams
    tr = build_flagship("cuda", "fp32", dropout=0.0, seed=42, encoder_dropout=0.0)
    tr.step({k: v.cuda() for k, v in tiny_batch(2, cfg=FULL, seed=31).items()})
    torch.cuda.synchronize()
    full = _grads(tr)
    floor = 1e-3 * max(abs(g).max() for g in full.values() if g is not None)
    worst = 0.0
    for k, g in full.items():
        if g is None:
            continue
        scale = max(abs(g).max(), floor)
        for r in range(world):
            e = abs(res[r][k] - g).max() / scale
            worst = max(worst, e)
            assert e < 2e-4, f"rank {r} {k}: {e:.2e}"
    print(f"full-size DP (2 ranks x 1 pair vs 1 x 2 pairs): worst gradient error {worst:.2e}, buckets {nb[0]}")


# ---- RCCL: ProcessGroupNCCL with one rank, the overlapped all-reduce forced on ----------------------
def _worker_nccl(port, q):
    import torch.distributed as dist
    _watchdog()
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        from mmfd.dp import GradAllReduce
        from mmfd.train import FusionTrainer, build_flagship
        from tests.smoke_impl import FULL, build_pair, tiny_batch
        out = {}
        # tiny models with 50 KB buckets: many buckets in flight on both encoder streams
        t_dp, _ = build_pair("fp32", dropout=0.0, seed=5)
        t_ref, _ = build_pair("fp32", dropout=0.0, seed=5)
        dp = GradAllReduce(bucket_mb=0.05, force=True)
        tr_dp = FusionTrainer(t_dp.text_encoder, t_dp.image_encoder, t_dp.head, lr=1e-3, precision="fp32", dp=dp)
        tr_ref = FusionTrainer(t_ref.text_encoder, t_ref.image_encoder, t_ref.head, lr=1e-3, precision="fp32")
        # full size with the default 32 MB buckets
        f_dp = build_flagship("cuda", "fp32", dropout=0.0, seed=42, dp=GradAllReduce(force=True))
        f_ref = build_flagship("cuda", "fp32", dropout=0.0, seed=42)
        for name, a, b, batches in (("tiny", tr_dp, tr_ref, [tiny_batch(4, seed=21), tiny_batch(4, seed=22)]),
                                    ("full", f_dp, f_ref, [tiny_batch(1, cfg=FULL, seed=41),
                                                           tiny_batch(1, cfg=FULL, seed=42)])):
            diffs = []
            for si, bt in enumerate(batches):
                la = a.step({k: v.cuda() for k, v in bt.items()})
                lb = b.step({k: v.cuda() for k, v in bt.items()})
                torch.cuda.synchronize()
                names = [n for m in (a.text_encoder, a.image_encoder, a.head) for n, _ in m.named_parameters()]
                for n, p, q_ in zip(names, a.params, b.params):
                    if (p.grad is None) != (q_.grad is None):
                        diffs.append((si, n, "grad None mismatch"))
                    elif p.grad is not None and not torch.equal(p.grad, q_.grad):
                        diffs.append((si, n, float((p.grad - q_.grad).abs().max() / p.grad.abs().max())))
            # bit for bit: every gradient kernel is deterministic (the embedding tables' scatter-add
            # sorts rows by id since round 5, csrc/embed_bwd.hip)
            same_grad = not diffs
            same_par = all(torch.equal(p, q_) for p, q_ in zip(a.params, b.params))
            same_loss = bool(torch.equal(la, lb))
            out[name] = (same_loss, same_grad, same_par, dict(a.dp.last_buckets), diffs[:12])
        out["backend"] = dist.get_backend()
        q.put(out)
    except BaseException:  # report instead of leaving the parent waiting on the queue
        import traceback
        q.put({"error": traceback.format_exc()})
        raise
    finally:
        dist.destroy_process_group()


def test_dp_nccl_world1_overlapped_allreduce():
    """the DP step on RCCL (ProcessGroupNCCL, world size 1, GradAllReduce forced active): the per-
    stream bucket packing, the async all_reduce on RCCL's stream and finish()'s wait + unpack run for
    two eager steps, tiny (many 50 KB buckets) and full size (default 32 MB buckets); a one-rank
    all-reduce is an identity, so losses, gradients and updated parameters equal the trainer
    without DP bit for bit (every gradient kernel is deterministic: the embedding tables' scatter-add
    sorts rows by id, csrc/embed_bwd.hip)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker_nccl, args=(_free_port(), q))
    p.start()
    out = _collect([p], q, 1)[0]
    assert "error" not in out, out.get("error")
    assert p.exitcode == 0
    assert out.pop("backend") == "nccl"
    for name, (same_loss, same_grad, same_par, nb, diffs) in out.items():
        assert same_loss and same_grad and same_par, (name, same_loss, same_grad, same_par, diffs)
        assert len(nb) == 2 and sum(nb.values()) >= 2, (name, nb)  # buckets from both encoder streams


def _worker_nccl_graph(port, q):
    """world-1 RCCL: a DP trainer whose whole step (with the bucketed all-reduce) is captured in a
    HIP graph vs the plain captured trainer, two replays on two batches each"""
    import torch.distributed as dist
    _watchdog()
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        from mmfd.dp import GradAllReduce
        from mmfd.train import FusionTrainer, build_flagship
        from tests.smoke_impl import FULL, build_pair, tiny_batch
        out = {}
        t_dp, _ = build_pair("fp32", dropout=0.1, seed=5, with_oracle=False)
        t_ref, _ = build_pair("fp32", dropout=0.1, seed=5, with_oracle=False)
        dp = GradAllReduce(bucket_mb=0.05, force=True)
        tr_dp = FusionTrainer(t_dp.text_encoder, t_dp.image_encoder, t_dp.head, lr=1e-3, precision="fp32", dp=dp)
        tr_ref = FusionTrainer(t_ref.text_encoder, t_ref.image_encoder, t_ref.head, lr=1e-3, precision="fp32")
        f_dp = build_flagship("cuda", "fp32", seed=42, dp=GradAllReduce(force=True))
        f_ref = build_flagship("cuda", "fp32", seed=42)
        for name, a, b, batches in (("tiny", tr_dp, tr_ref, [tiny_batch(4, seed=21), tiny_batch(4, seed=22),
                                                             tiny_batch(4, seed=23)]),
                                    ("full", f_dp, f_ref, [tiny_batch(1, cfg=FULL, seed=41),
                                                           tiny_batch(1, cfg=FULL, seed=42),
                                                           tiny_batch(1, cfg=FULL, seed=43)])):
            static_a = {k: v.cuda() for k, v in batches[0].items()}
            static_b = {k: v.cuda() for k, v in batches[0].items()}
            a.capture(static_a, warmup=1)
            b.capture(static_b, warmup=1)
            names = [n for m in (a.text_encoder, a.image_encoder, a.head) for n, _ in m.named_parameters()]
            ok = []
            for bt in batches[1:]:
                la = a.replay({k: v.cuda() for k, v in bt.items()}).clone()
                lb = b.replay({k: v.cuda() for k, v in bt.items()}).clone()
                torch.cuda.synchronize()
                bad = []
                for n, p, q_ in zip(names, a.params, b.params):
                    tol = 0.0  # bit for bit (deterministic kernels, csrc/embed_bwd.hip)
                    for what, x, y in (("grad", p.grad, q_.grad), ("param", p.detach(), q_.detach())):
                        if (x is None) != (y is None):
                            bad.append((n, what, "None"))
                        elif x is not None:
                            d = float((x - y).abs().max())
                            if d > tol * max(1.0, float(y.abs().max())):
                                bad.append((n, what, d, float(y.abs().max())))
                ok.append((float((la - lb).abs().max()), bad[:8]))
            buckets = dict(a.dp.last_buckets)
            # the bench's self-check of a captured DP step (one more replay, then the cross-rank
            # checksum of gradients + parameters; trivially equal with one rank, run for the code path)
            out[name] = (ok, buckets, a.verify_capture())
            a.release_graph()
            b.release_graph()
        q.put(out)
    except BaseException:
        import traceback
        q.put({"error": traceback.format_exc()})
        raise
    finally:
        dist.destroy_process_group()


def test_dp_nccl_world1_graph_captured_step():
    """the data-parallel step captured as ONE HIP graph — forward, backward with the
    per-stream bucket packs and the RCCL all_reduce kernels, finish()'s wait + unpack, AdamW — on
    ProcessGroupNCCL (RCCL) with one rank. Replayed on new batches it must equal the plain captured
    step (no DP) in losses, gradients and updated parameters, bit for bit (deterministic kernels:
    csrc/embed_bwd.hip), tiny with 50 KB buckets and full size
    with the default 32 MB buckets, dropout on. Since round 5 the captured all-reduces run on the DP
    object's dedicated capture group in the thread-local capture mode (no quiesce sleep before the
    capture; mmfd.dp), and the bench's cross-rank self-check (verify_capture) runs on it."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker_nccl_graph, args=(_free_port(), q))
    p.start()
    out = _collect([p], q, 1)[0]
    assert "error" not in out, out.get("error")
    assert p.exitcode == 0
    for name, (steps, nb, verified) in out.items():
        for lerr, bad in steps:
            assert lerr == 0.0 and not bad, (name, lerr, bad)
        assert len(nb) == 2 and sum(nb.values()) >= 2, (name, nb)
        assert verified, name
