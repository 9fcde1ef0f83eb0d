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
