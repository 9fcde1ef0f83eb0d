"""Sharded retrieval merge: per-shard exact top-k candidates, concatenated in shard
order and reduced by one more exact top-k, equal the single-process top-k — ties resolved to the
lower global index — at every shard count, including shards with fewer rows than k.
The device top-k is replaced here by a stable host sort with the same contract as mmfd_topk."""
import torch

from mmfd.retrieval import merge_topk


def _topk_host(scores, k):
    """mmfd_topk's contract: k largest per row, descending, ties -> lower index; -inf / -1 padding"""
    Q, N = scores.shape
    order = torch.sort(-scores, dim=1, stable=True).indices[:, :k]
    vals = torch.gather(scores, 1, order)
    if order.shape[1] < k:
        pad = k - order.shape[1]
        vals = torch.cat([vals, torch.full((Q, pad), float("-inf"))], 1)
        order = torch.cat([order, torch.full((Q, pad), -1, dtype=torch.int64)], 1)
    return vals, order


def test_merge_equals_global_topk_with_ties():
    g = torch.Generator().manual_seed(5)
    Q, N, k = 3, 37, 9
    scores = (torch.randint(0, 6, (Q, N), generator=g).float() / 5.0)  # many ties
    ref_v, ref_i = _topk_host(scores, k)
    for world in (1, 2, 3, 5, 8):
        cands = []
        for r in range(world):
            lo, hi = N * r // world, N * (r + 1) // world
            kl = min(k, hi - lo)
            v = torch.full((Q, k), float("-inf"))
            i = torch.full((Q, k), -1, dtype=torch.int64)
            if kl:
                lv, li = _topk_host(scores[:, lo:hi], kl)
                v[:, :kl], i[:, :kl] = lv, li + lo
            cands.append((v, i))
        mv, mi = merge_topk(cands, k, topk=_topk_host)
        assert torch.equal(mv, ref_v) and torch.equal(mi, ref_i), world
