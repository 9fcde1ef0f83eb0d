"""Data-parallel gradient averaging (mmfd.dp.GradAllReduce) over gloo, world_size 2, on the CPU.

The HIP pack/unpack kernels are swapped for torch copies here (no GPU in this container); the
bucketing, the asynchronous all-reduce and the 1/world scaling are the code under test.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _pack(g, dst):
    dst.copy_(g.reshape(-1).float())


def _unpack(src, g, scale):
    g.copy_((src * scale).view(g.shape))


def _worker(rank, world, port, bucket_mb, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mmfd.dp import GradAllReduce

        shapes = [(7, 5), (300,), (64, 33), (1,), (129, 3)]
        params = []
        for i, s in enumerate(shapes):
            p = torch.zeros(s, requires_grad=True)
            g = torch.Generator().manual_seed(1000 * rank + i)
            p.grad = torch.randn(s, generator=g)
            params.append(p)
        params.append(torch.zeros(3, requires_grad=True))  # no grad: skipped
        GradAllReduce(bucket_mb=bucket_mb, pack=_pack, unpack=_unpack).allreduce_grads(params)
        res = [p.grad.clone() if p.grad is not None else None for p in params]
        # overlapped protocol: layers report finished gradients in backward order (hook_for maps
        # names to parameters); the averages land in .grad at finish()
        m = torch.nn.Sequential(torch.nn.Linear(5, 7), torch.nn.Linear(7, 300))
        grads = {}
        for i, (n, p) in enumerate(m.named_parameters()):
            grads[n] = torch.randn(p.shape, generator=torch.Generator().manual_seed(100 * rank + i))
            p.grad = grads[n].clone()
        dp = GradAllReduce(bucket_mb=bucket_mb, pack=_pack, unpack=_unpack)
        hook = dp.hook_for(m)
        dp.begin()
        hook(["1.weight", "1.bias"], grads)
        hook(["0.weight", "0.bias"], grads)
        dp.finish()
        res += [p.grad.clone() for p in m.parameters()]
        # plain numpy: torch tensors travel as shared-memory fds that vanish when the worker exits
        q.put((rank, [r.numpy() if r is not None else None for r in res]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,bucket_mb", [(2, 64.0), (2, 0.001), (4, 0.001), (8, 0.001)])
def test_grad_allreduce_gloo_world2(world, bucket_mb):
    """one bucket / many small buckets; world 4 and 8 rehearse the node layout bench.py --gpus N
    launches (gloo on the CPU: the 8-GPU run itself is the driver's)"""
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, bucket_mb, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    res = {k: [torch.from_numpy(a) if a is not None else None for a in v] for k, v in res.items()}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    shapes = [(7, 5), (300,), (64, 33), (1,), (129, 3)]
    for i, s in enumerate(shapes):
        want = sum(torch.randn(s, generator=torch.Generator().manual_seed(1000 * r + i)) for r in range(world)) / world
        for r in range(world):
            torch.testing.assert_close(res[r][i], want, rtol=1e-6, atol=1e-6)
    assert all(res[r][5] is None for r in range(world))
    m = torch.nn.Sequential(torch.nn.Linear(5, 7), torch.nn.Linear(7, 300))
    for i, (n, p) in enumerate(m.named_parameters()):
        want = sum(torch.randn(p.shape, generator=torch.Generator().manual_seed(100 * r + i)) for r in range(world)) / world
        for r in range(world):
            torch.testing.assert_close(res[r][6 + i], want, rtol=1e-6, atol=1e-6)


def _train_worker(rank, world, port, q):
    """Replicas initialised from DIFFERENT seeds, different data per rank: after the rank-0
    broadcast and two averaged steps every rank must hold bitwise-identical parameters."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mmfd.dp import GradAllReduce

        torch.manual_seed(100 + rank)
        m = torch.nn.Sequential(torch.nn.Linear(5, 16), torch.nn.GELU(), torch.nn.Linear(16, 3))
        dp = GradAllReduce(bucket_mb=0.0005, pack=_pack, unpack=_unpack)
        dp.broadcast_params(list(m.parameters()))
        init = [p.detach().clone().numpy() for p in m.parameters()]
        opt = torch.optim.AdamW(m.parameters(), lr=1e-2)
        g = torch.Generator().manual_seed(7 + rank)
        for _ in range(2):
            opt.zero_grad(set_to_none=True)
            x = torch.randn(8, 5, generator=g)
            y = torch.randint(0, 3, (8,), generator=g)
            torch.nn.functional.cross_entropy(m(x), y).backward()
            dp.allreduce_grads(list(m.parameters()))
            opt.step()
        q.put((rank, init, [p.detach().clone().numpy() for p in m.parameters()]))
    finally:
        dist.destroy_process_group()


def test_replicas_from_different_seeds_stay_identical():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_train_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, init, final = q.get(timeout=120)
        res[r] = (init, final)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    torch.manual_seed(100)  # rank 0's initialisation is the one every rank must hold
    m0 = torch.nn.Sequential(torch.nn.Linear(5, 16), torch.nn.GELU(), torch.nn.Linear(16, 3))
    for a, b, p0 in zip(res[0][0], res[1][0], m0.parameters()):
        assert (a == b).all() and (a == p0.detach().numpy()).all()
    for a, b in zip(res[0][1], res[1][1]):
        assert (a == b).all()
    assert any((a != b).any() for a, b in zip(res[0][0], res[0][1]))  # and training moved them


def _check_worker(rank, world, port, q):
    """mmfd.dp.state_checksum / GradAllReduce.consistent and mmfd.train.capture_dp_step over gloo:
    identical tensors agree, a one-bit difference on one rank does not, and a captured step whose
    replay leaves the ranks different (or whose capture failed on one rank) is released on EVERY rank."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mmfd.dp import GradAllReduce, state_checksum
        from mmfd.train import capture_dp_step

        dp = GradAllReduce(pack=_pack, unpack=_unpack)
        g = torch.Generator().manual_seed(3)
        same = [torch.randn(17, 5, generator=g), None, torch.randn(300, generator=g).bfloat16(),
                torch.arange(7, dtype=torch.int64)]
        res = {"same": dp.consistent(same)}
        flipped = [t.clone() if t is not None else None for t in same]
        if rank == 1:  # one bit of one element on one rank
            flipped[0].view(torch.int32)[3, 2] ^= 1
        res["flipped"] = dp.consistent(flipped)
        swapped = [same[2], None, same[0], same[3]] if rank == 1 else same  # same tensors, other order
        res["swapped"] = dp.consistent(swapped)
        res["sum_order_free"] = bool(torch.equal(state_checksum([same[0]]), state_checksum([same[0].flip(0).flip(0)])))

        class FakeTrainer:
            """capture / verify / release as FusionTrainer; `mismatch` makes rank 1's replay differ"""
            def __init__(self, fail_capture=False, mismatch=False):
                self.fail_capture, self.mismatch, self.released, self.dp = fail_capture, mismatch, False, dp
                self.p = torch.ones(4)

            def capture(self, batch, warmup):
                if self.fail_capture and rank == 0:
                    raise RuntimeError("capture refused")

            def verify_capture(self):
                if self.mismatch and rank == 1:
                    self.p[0] += 1.0  # the all-reduce "did not run": rank 1's state differs
                return self.dp.consistent([self.p])

            def release_graph(self):
                self.released = True

            def resync_state(self, src=0):
                self.dp.broadcast_tensors([self.p], src=src)

        for name, kw in (("ok", {}), ("mismatch", {"mismatch": True}), ("capture_fail", {"fail_capture": True})):
            t = FakeTrainer(**kw)
            graphed, msg = capture_dp_step(t, None, 1, "cpu", log=lambda m: None)
            res["dp_" + name] = (graphed, t.released, msg, dp.consistent([t.p]))
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def test_cross_rank_checksum_and_capture_fallback_gloo_world2():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_check_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        got = res[r]
        assert got["same"] is True and got["flipped"] is False and got["swapped"] is False
        assert got["sum_order_free"]
        assert got["dp_ok"][:2] == (True, False), got["dp_ok"]
        # the mismatch branch: both ranks release the graph and run eager steps, whichever differed
        assert got["dp_mismatch"][:2] == (False, True) and "MISMATCH" in got["dp_mismatch"][2], got["dp_mismatch"]
        # ... and the state the verifying replay left diverged is rank 0's again on every rank
        assert got["dp_mismatch"][3] is True and got["dp_ok"][3] is True, got["dp_mismatch"]
        assert got["dp_capture_fail"][:2] == (False, True), got["dp_capture_fail"]
