"""Evidence retrieval scoring on HIP (csrc/retrieval.hip, mmfd.retrieval) against the CPU oracle
(oracle/retrieval.py, float64).

Tolerances: scores of fp32 / bf16 / fp16 corpora (exactly representable inputs, fp32 accumulation)
within 2e-6 absolute of the float64 oracle (|score| <= 1); fp16-rounded scores within one fp16 ulp.
Top-k is exact: the same values and the same indices as a stable descending sort (ties -> lower
index), at every size including ragged segment tails and k > N. Search results equal the oracle's
distinct-score filter whenever the oracle's consecutive scores are separated by more than the
score tolerance (random features; planted duplicate rows give bit-identical scores on both sides).
"""
import numpy as np
import pytest
import torch

import mmfd  # noqa: F401
from mmfd import kernels as K
from mmfd.retrieval import CorpusIndex, dedupe_by_score, semantic_search
from oracle.retrieval import cosine_normalized, cosine_pair, ranked, retrieve_unique

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("Q,N,D", [(1, 1, 8), (3, 1000, 2048), (8, 517, 768), (11, 4099, 64), (1, 41256, 2048)])
def test_cosine_scores_vs_oracle(dtype, Q, N, D):
    g = torch.Generator().manual_seed(N + D)
    c = torch.randn(N, D, generator=g).to(dtype)
    q = torch.randn(Q, D, generator=g)
    if N > 5:
        c[3] = 0  # zero row: eps clamp
    s = K.cosine_scores(q.to(DEV), c.to(DEV), mode=K.COS_PAIR, eps=1e-6)
    ref = cosine_pair(q.numpy(), c.float().numpy(), eps=1e-6)
    assert np.abs(s.cpu().numpy() - ref).max() < 2e-6
    s2 = K.cosine_scores(q.to(DEV), c.to(DEV), mode=K.COS_NORMALIZED, eps=1e-12)
    ref2 = cosine_normalized(q.numpy(), c.float().numpy())
    assert np.abs(s2.cpu().numpy() - ref2).max() < 2e-6
    s3 = K.cosine_scores(q.to(DEV), c.to(DEV), mode=K.COS_NORMALIZED | K.COS_ROUND_F16, eps=1e-12)
    ulp = np.abs(ref2.astype(np.float16).astype(np.float64) - ref2).max() * 2 + 1e-7
    assert np.abs(s3.cpu().numpy() - ref2).max() <= ulp
    assert np.array_equal(s3.cpu().numpy(), s3.cpu().numpy().astype(np.float16).astype(np.float32))


@pytest.mark.parametrize("N", [1, 7, 4096, 4097, 41256, 100003])
@pytest.mark.parametrize("k", [1, 5, 64, 250, 2048])
def test_topk_exact_with_ties(N, k):
    g = torch.Generator().manual_seed(N * 7 + k)
    Q = 3
    # quantised scores -> many exact ties; include negatives, -inf-free
    s = (torch.randint(-50, 50, (Q, N), generator=g).float() / 16.0)
    val, idx = K.topk(s.to(DEV), k)
    val, idx = val.cpu().numpy(), idx.cpu().numpy()
    for q in range(Q):
        order = ranked(s[q].numpy())[:k]
        kk = min(k, N)
        assert np.array_equal(idx[q, :kk], order), (q, idx[q, :10], order[:10])
        assert np.array_equal(val[q, :kk], s[q].numpy()[order])
        if k > N:
            assert (idx[q, N:] == -1).all() and np.isneginf(val[q, N:]).all()


def test_topk_strided_rows_and_errors():
    s = torch.randn(4, 300, device=DEV)
    big = torch.empty(4, 512, device=DEV)
    big[:, :300] = s
    v1, i1 = K.topk(big[:, :300], 10)
    v2, i2 = K.topk(s, 10)
    assert torch.equal(v1, v2) and torch.equal(i1, i2)
    with pytest.raises(RuntimeError):
        K.topk(s, 4096)


def test_image_search_matches_reference_semantics():
    """CorpusIndex.search in the image mode == oracle: nn.CosineSimilarity(eps=1e-6) scores, stable
    descending order, distinct-score filter; planted duplicates collapse to their first row."""
    g = torch.Generator().manual_seed(11)
    N, D = 41256, 2048
    feats = torch.randn(N, D, generator=g).abs()  # ResNet features are post-ReLU averages: non-negative
    q = torch.randn(2, D, generator=g).abs()
    # plant duplicates of strong matches of query 0 (identical rows -> identical scores)
    best = torch.topk(torch.nn.functional.cosine_similarity(feats, q[0:1], dim=1, eps=1e-6), 6).indices
    for j, src in enumerate(best.tolist()):
        feats[100 + 3 * j] = feats[src]
        feats[30000 + j] = feats[src]
    ids = [f"img_{i}.jpg" for i in range(N)]
    index = CorpusIndex(feats, ids=ids, mode="pair", eps=1e-6)
    got = index.search(q.to(DEV), top_k=50)
    ref_scores = cosine_pair(q.numpy(), feats.numpy(), eps=1e-6)
    for qi in range(2):
        ref = retrieve_unique(ref_scores[qi], 50)
        pos = {name: i for i, name in enumerate(ids)}
        picked = [pos[p] for p, _ in got[qi]]
        assert len(picked) == 50
        # rank by rank, the pick's exact score equals the oracle's up to fp32 rounding: the lists
        # agree except for swaps inside near-ties the fp32 scores cannot order
        np.testing.assert_allclose(ref_scores[qi][picked], [v for _, v in ref], atol=4e-6)
        np.testing.assert_allclose([v for _, v in got[qi]], ref_scores[qi][picked], atol=2e-6)
        gaps = np.abs(np.diff([v for _, v in ref]))
        agree = [a == b for (a, _), b in zip(ref, picked)]
        assert all(ok or gaps[max(i - 1, 0):i + 1].min() < 1e-5 for i, ok in enumerate(agree))
    # every planted duplicate was filtered in favour of the lowest corpus index
    chosen = {p for p, _ in got[0]}
    for j, src in enumerate(best.tolist()):
        group = sorted({src, 100 + 3 * j, 30000 + j})
        assert [ids[i] in chosen for i in group] == [True] + [False] * (len(group) - 1), (j, group)


def test_search_needs_more_candidates_than_top_k():
    """many exact duplicates: the distinct filter must widen the candidate list"""
    D = 64
    base = torch.randn(5, D)
    feats = base.repeat_interleave(40, dim=0)  # 200 rows, 5 distinct scores per query
    index = CorpusIndex(feats, mode="pair")
    q = torch.randn(1, D)
    got = index.search(q.to(DEV), top_k=5)[0]
    ref = retrieve_unique(cosine_pair(q.numpy(), feats.numpy())[0], 5)
    assert [i for i, _ in got] == [i for i, _ in ref]
    vals = torch.tensor([0.9, 0.9, 0.8]), torch.tensor([3, 4, 9])
    assert dedupe_by_score(vals[0].tolist(), vals[1].tolist(), 5) == ([(3, pytest.approx(0.9)), (9, pytest.approx(0.8))], True)


def test_semantic_search_format_and_fp16_scores():
    """util.semantic_search: [{'corpus_id', 'score'}] per query, sorted, cos_sim of fp16 embeddings"""
    g = torch.Generator().manual_seed(5)
    corpus = torch.randn(35000, 768, generator=g).half()
    q = torch.randn(2, 768, generator=g).half()
    hits = semantic_search(q.to(DEV), corpus.to(DEV), top_k=25)
    ref = cosine_normalized(q.float().numpy(), corpus.float().numpy())
    for qi in range(2):
        assert len(hits[qi]) == 25
        sc = [h["score"] for h in hits[qi]]
        assert sc == sorted(sc, reverse=True)
        top = ranked(ref[qi])[:25]
        # fp16-rounded scores: the same set of hits up to ties created by the rounding
        assert np.abs(np.array(sc) - ref[qi][top]).max() < 1e-3
        assert set(h["corpus_id"] for h in hits[qi][:10]) <= set(ranked(ref[qi])[:40].tolist())


def test_image_corpus_retrieve_similar_images(tmp_path):
    from PIL import Image
    from mmfd.evidence import ImageCorpus, ImageSimilarity, ResNet
    rng = np.random.default_rng(1)
    for i in range(6):
        Image.fromarray(rng.integers(0, 255, (48, 40 + i, 3), dtype=np.uint8)).save(tmp_path / f"img{i}.png")
    Image.open(tmp_path / "img2.png").save(tmp_path / "img2_copy.png")  # identical image -> identical score
    ext = ImageSimilarity(model=ResNet((1, 1, 1, 1), 8), precision="fp32")
    corpus = ImageCorpus(str(tmp_path / "feats.npz"), extractor=ext)
    corpus.create_feature_corpus(str(tmp_path))
    got = corpus.retrieve_similar_images(str(tmp_path / "img2.png"), top_k=50)
    paths = list(corpus.feature_dict)
    feats = torch.stack([corpus.feature_dict[p] for p in paths]).numpy()
    qf = ext.extract_features(str(tmp_path / "img2.png")).numpy()[None]
    ref = retrieve_unique(cosine_pair(qf, feats)[0], 50)
    assert [p for p, _ in got] == [paths[i] for i, _ in ref]
    assert len(got) == 6  # 7 images, the copy shares img2's score
    assert got[0][0].endswith("img2.png") and abs(got[0][1] - 1.0) < 1e-5
