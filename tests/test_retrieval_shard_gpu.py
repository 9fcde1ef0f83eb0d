"""Sharded corpus retrieval on the HIP path: 2 ranks (gloo, both on cuda:0 — the box
has one GPU) each keep half of the corpus rows, search the same queries with the local
cosine + exact top-k kernels, exchange the k candidates and merge: the hits (indices and scores,
distinct-score filter on) must equal a single-process CorpusIndex.search over the whole corpus,
exactly. Scores are quantised so that ties across the shard boundary occur."""
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


def _data():
    g = torch.Generator().manual_seed(11)
    feats = torch.randint(1, 4, (301, 64), generator=g).float()  # few distinct directions: tied scores
    q = torch.randint(1, 4, (5, 64), generator=g).float()
    return feats, q


def _worker(rank, world, port, q):
    import torch.distributed as dist
    from tests.mp_util import watchdog
    watchdog()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mmfd.retrieval import ShardedCorpusIndex
        feats, queries = _data()
        idx = ShardedCorpusIndex(feats, mode="pair", eps=1e-6, device="cuda")
        hits = idx.search(queries.cuda(), 12)
        v, i = idx.topk(queries.cuda(), 40)
        q.put((rank, hits, v.cpu(), i.cpu()))
    finally:
        dist.destroy_process_group()


def test_sharded_search_equals_single_process():
    from mmfd.retrieval import CorpusIndex
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    from tests.mp_util import collect
    out = {}
    for r, hits, v, i in collect(procs, q, world):
        out[r] = (hits, v, i)
    assert all(p.exitcode == 0 for p in procs)
    feats, queries = _data()
    ref = CorpusIndex(feats, mode="pair", eps=1e-6, device="cuda")
    ref_hits = ref.search(queries.cuda(), 12)
    rv, ri = ref.topk(queries.cuda(), 40)
    for r in range(world):
        hits, v, i = out[r]
        assert hits == ref_hits
        assert torch.equal(v, rv.cpu()) and torch.equal(i, ri.cpu())
