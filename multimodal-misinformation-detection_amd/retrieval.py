"""Evidence retrieval scoring on HIP.

Reference semantics, kept exactly:
  * image search, ImageCorpus.retrieve_similar_images (src/evidence/im2im_retrieval.py:80-106):
    nn.CosineSimilarity(dim=1, eps=1e-6) of the query against every corpus feature, sorted by
    score descending (Python's stable sort: equal scores keep corpus insertion order), then the
    first `top_k` entries with pairwise-distinct scores ("filter out identical images");
  * text search, the bi-encoder stage of SemanticSimilarity.search
    (src/evidence/text2text_retrieval.py:49-66): sentence_transformers.util.semantic_search,
    i.e. cos_sim of L2-normalised fp16 embeddings and the top-k hits per query as
    [{"corpus_id": i, "score": s}, ...] sorted by score.

Both run as two kernels over a corpus that stays resident in HBM (`CorpusIndex`): one HBM-bound
pass computing the scores of a query batch (`mmfd_cosine_scores`) and an exact top-k
(`mmfd_topk`). Only the final, already sorted candidate list comes back to the host, where the
distinct-score filter walks it (it needs at most a few more candidates than `top_k`; the
candidate count grows until the filter is satisfied or the corpus is exhausted).
The MiniLM cross-encoder re-ranking of text2text_retrieval.py:68-118 and the SemanticSimilarity
class are in mmfd.rerank; `dedupe_by_score` is the shared distinct-score filter.
"""
from __future__ import annotations

import torch

from . import kernels as K

MAX_CANDIDATES = 2048  # mmfd_topk's k limit


def dedupe_by_score(values, indices, top_k):
    """The reference's distinct-score filter (im2im_retrieval.py:98-106,
    text2text_retrieval.py:107-118) over one query's sorted candidates -> [(index, score)] and
    whether the candidate list ran out before `top_k` distinct scores were found."""
    seen, out = set(), []
    for s, i in zip(values, indices):
        if i < 0:
            return out, False
        if s not in seen:
            seen.add(s)
            out.append((int(i), float(s)))
        if len(out) == top_k:
            return out, False
    return out, True


class CorpusIndex:
    """A device-resident embedding corpus [N, D] (fp32 / bf16 / fp16) with cosine search.

    mode "pair": nn.CosineSimilarity(dim=1, eps) (image features, eps 1e-6);
    mode "normalized": util.cos_sim (eps 1e-12), `round_f16` rounds scores to fp16 as the
    reference's fp16 embeddings produce them."""

    def __init__(self, embeddings, ids=None, device="cuda", mode="pair", eps=None, round_f16=False):
        if not torch.is_tensor(embeddings):
            embeddings = torch.as_tensor(embeddings)
        self.emb = embeddings.to(device).contiguous()
        self.ids = list(ids) if ids is not None else None
        self.mode = (K.COS_PAIR if mode == "pair" else K.COS_NORMALIZED) | (K.COS_ROUND_F16 if round_f16 else 0)
        self.eps = eps if eps is not None else (1e-6 if mode == "pair" else 1e-12)

    def __len__(self):
        return self.emb.shape[0]

    def scores(self, queries):
        """fp32 [Q, N] scores on the device"""
        q = queries.to(self.emb.device)
        return K.cosine_scores(q, self.emb, mode=self.mode, eps=self.eps)

    def topk(self, queries, k):
        """(values [Q, k], indices [Q, k]) on the device, descending, ties -> lower index"""
        k = min(k, len(self))
        return K.topk(self.scores(queries), k)

    def search(self, queries, top_k, unique=True):
        """Per query, [(id_or_index, score)] of the `top_k` best entries (distinct scores when
        `unique`, as the reference filters them)."""
        if queries.dim() == 1:
            queries = queries.unsqueeze(0)
        s = self.scores(queries)
        n = len(self)
        want = min(n, top_k if not unique else max(top_k + 8, 2 * top_k))
        results = [None] * queries.shape[0]
        todo = list(range(queries.shape[0]))
        while todo:
            kk = min(want, n, MAX_CANDIDATES)
            vals, idx = K.topk(s[todo], kk)
            vals, idx = vals.cpu().tolist(), idx.cpu().tolist()
            again = []
            for row, q in enumerate(todo):
                if unique:
                    hits, short = dedupe_by_score(vals[row], idx[row], top_k)
                    if short and kk < n:
                        if kk == MAX_CANDIDATES:
                            raise RuntimeError(f"more than {MAX_CANDIDATES} candidates needed for {top_k} distinct scores")
                        again.append(q)
                        continue
                else:
                    hits = [(int(i), float(v)) for v, i in zip(vals[row][:top_k], idx[row][:top_k]) if i >= 0]
                results[q] = [(self.ids[i] if self.ids is not None else i, v) for i, v in hits]
            todo, want = again, want * 4
        return results


def semantic_search(query_embeddings, corpus_embeddings, top_k=10, round_f16=True):
    """sentence_transformers.util.semantic_search on HIP: per query, the top_k corpus entries by
    cos_sim as [{"corpus_id": i, "score": s}] sorted by decreasing score (ties: lower id first)."""
    index = corpus_embeddings if isinstance(corpus_embeddings, CorpusIndex) else \
        CorpusIndex(corpus_embeddings, device=query_embeddings.device if query_embeddings.is_cuda else "cuda",
                    mode="normalized", round_f16=round_f16)
    q = query_embeddings if query_embeddings.dim() == 2 else query_embeddings.unsqueeze(0)
    vals, idx = index.topk(q.float(), top_k)
    vals, idx = vals.cpu().tolist(), idx.cpu().tolist()
    return [[{"corpus_id": int(i), "score": float(v)} for v, i in zip(vr, ir) if i >= 0] for vr, ir in zip(vals, idx)]


def merge_topk(candidates, k, topk=None):
    """Global top-k from per-shard candidate lists: `candidates` = [(values [Q, k_r]
    fp32, global indices [Q, k_r] int64)] in shard order, each sorted descending with ties by lower
    index and padded with -inf / -1. Concatenated in shard order (contiguous shards: a lower shard
    holds lower global indices), an exact top-k over the positions with ties to the lower position is
    the single-process answer. `topk` (default mmfd_topk) -> (values [Q, k], global indices [Q, k])."""
    vals = torch.cat([v for v, _ in candidates], dim=1).contiguous()
    gidx = torch.cat([i for _, i in candidates], dim=1)
    k = min(k, vals.shape[1])
    mv, pos = (topk or K.topk)(vals, k)
    gi = torch.gather(gidx, 1, pos.clamp(min=0))
    return mv, torch.where(pos >= 0, gi, torch.full_like(gi, -1))


class ShardedCorpusIndex:
    """A corpus whose rows are split contiguously over the ranks of a process group (SURVEY §8(e):
    each GPU keeps only its shard resident). topk(): every rank scores the same queries against its
    shard and keeps its exact local top-k (`mmfd_cosine_scores` + `mmfd_topk`), one all_gather moves
    the k candidates (scores + global row ids) of every rank, and `merge_topk` reduces them — every
    rank ends with the single-process answer, ties included. Collective: all ranks must call with the
    same query batch and k."""

    def __init__(self, embeddings, ids=None, device="cuda", mode="pair", eps=None, round_f16=False, group=None,
                 local_shard=False):
        import torch.distributed as dist
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        if local_shard:  # `embeddings` is already this rank's contiguous shard
            sizes = self._gather_ints(embeddings.shape[0])
            self.offset, self.n_total = sum(sizes[:self.rank]), sum(sizes)
            shard = embeddings
        else:
            n = embeddings.shape[0]
            lo = n * self.rank // self.world
            hi = n * (self.rank + 1) // self.world
            self.offset, self.n_total = lo, n
            shard = embeddings[lo:hi]
        self.ids = list(ids) if ids is not None else None
        self.local = CorpusIndex(shard, device=device, mode=mode, eps=eps, round_f16=round_f16)

    def _gather_ints(self, x):
        import torch.distributed as dist
        if self.world == 1:
            return [int(x)]
        dev = "cuda" if dist.get_backend(self.group) == "nccl" else "cpu"
        t = torch.tensor([int(x)], dtype=torch.int64, device=dev)
        out = [torch.zeros_like(t) for _ in range(self.world)]
        dist.all_gather(out, t, group=self.group)
        return [int(v.item()) for v in out]

    def __len__(self):
        return self.n_total

    def topk(self, queries, k):
        import torch.distributed as dist
        k = min(k, self.n_total)
        q = queries.to(self.local.emb.device)
        Q = q.shape[0]
        kl = min(k, len(self.local))
        vals = torch.full((Q, k), float("-inf"), device=q.device)
        gidx = torch.full((Q, k), -1, dtype=torch.int64, device=q.device)
        if kl > 0:
            v, i = self.local.topk(q, kl)
            vals[:, :kl] = v
            gidx[:, :kl] = torch.where(i >= 0, i + self.offset, i)
        if self.world == 1:
            return vals, gidx
        dev = vals.device
        if dist.get_backend(self.group) != "nccl":  # gloo gathers host tensors only
            vals, gidx = vals.cpu(), gidx.cpu()
        vs = [torch.empty_like(vals) for _ in range(self.world)]
        gs = [torch.empty_like(gidx) for _ in range(self.world)]
        dist.all_gather(vs, vals, group=self.group)
        dist.all_gather(gs, gidx, group=self.group)
        return merge_topk([(v.to(dev), g.to(dev)) for v, g in zip(vs, gs)], k)

    def search(self, queries, top_k, unique=True):
        """CorpusIndex.search over the sharded corpus (collective; every rank returns the same hits)"""
        if queries.dim() == 1:
            queries = queries.unsqueeze(0)
        n = self.n_total
        want = min(n, top_k if not unique else max(top_k + 8, 2 * top_k))
        while True:
            kk = min(want, n, MAX_CANDIDATES)
            vals, idx = self.topk(queries, kk)
            vals, idx = vals.cpu().tolist(), idx.cpu().tolist()
            results, short_any = [], False
            for row in range(len(vals)):
                if unique:
                    hits, short = dedupe_by_score(vals[row], idx[row], top_k)
                    short_any |= short and kk < n
                else:
                    hits = [(int(i), float(v)) for v, i in zip(vals[row][:top_k], idx[row][:top_k]) if i >= 0]
                results.append([(self.ids[i] if self.ids is not None else i, v) for i, v in hits])
            if not short_any:
                return results
            if kk == MAX_CANDIDATES:
                raise RuntimeError(f"more than {MAX_CANDIDATES} candidates needed for {top_k} distinct scores")
            want *= 4
