"""CPU oracle for evidence retrieval scoring (TEST INFRASTRUCTURE ONLY: imported by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline, never by the product path).

Restates, in numpy float64:
  * nn.CosineSimilarity(dim=1, eps=1e-6) per corpus entry + sorted(reverse=True) + the
    distinct-score filter of ImageCorpus.retrieve_similar_images
    (src/evidence/im2im_retrieval.py:38-42, 80-106);
  * sentence_transformers.util.cos_sim / semantic_search as called at
    src/evidence/text2text_retrieval.py:55-66 (sentence-transformers 3.3.1 is not installed here:
    its published algorithm is restated — normalise each embedding by max(||x||, 1e-12), dot,
    top-k by score).
Parity of the product path with this oracle is pinned by tests/test_retrieval_gpu.py; the oracle
itself is pinned against torch's own nn.CosineSimilarity / F.normalize on CPU in
tests/test_oracle_golden.py (the reference's retrieval code needs torchvision / h5py /
sentence-transformers, none importable here).
"""
import numpy as np


def cosine_pair(queries, corpus, eps=1e-6):
    """nn.CosineSimilarity(dim=1, eps): x.y / sqrt(max(|x|^2 |y|^2, eps^2)) -> [Q, N] float64"""
    q = np.asarray(queries, np.float64)
    c = np.asarray(corpus, np.float64)
    dot = q @ c.T
    qq = (q * q).sum(1)[:, None]
    cc = (c * c).sum(1)[None, :]
    return dot / np.sqrt(np.maximum(qq * cc, eps * eps))


def cosine_normalized(queries, corpus, eps=1e-12):
    """util.cos_sim: normalize(x) . normalize(y) with F.normalize's max(||x||, eps)"""
    q = np.asarray(queries, np.float64)
    c = np.asarray(corpus, np.float64)
    qn = q / np.maximum(np.linalg.norm(q, axis=1, keepdims=True), eps)
    cn = c / np.maximum(np.linalg.norm(c, axis=1, keepdims=True), eps)
    return qn @ cn.T


def ranked(scores):
    """indices of one query's scores in the reference's order: descending score, stable (lower
    index first among equal scores) — sorted(items, key=score, reverse=True) keeps insertion order
    for ties, exactly like a stable descending sort"""
    s = np.asarray(scores)
    return np.argsort(-s, kind="stable")


def retrieve_unique(scores, top_k):
    """the distinct-score filter over the ranked list (im2im_retrieval.py:98-106)"""
    seen, out = set(), []
    for i in ranked(scores):
        v = float(scores[i])
        if v not in seen:
            seen.add(v)
            out.append((int(i), v))
        if len(out) == top_k:
            break
    return out
