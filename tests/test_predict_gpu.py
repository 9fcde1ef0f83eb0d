"""Single-pair inference (evaluate.py:95-192) on the HIP path: the captured
HIP-graph forward equals the eager forward bit for bit, both match the CPU oracle (fp32 logits
within north_star's 1e-3 abs; bf16 within 5e-2), and `evaluate` returns the reference's per-path
labels (softmax -> argmax over idx_to_label, evaluate.py:82,169-192). Text is padded to
max_length=512 as the reference's tokenizer call does (evaluate.py:112-126)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _pair(L_real, seed):
    g = torch.Generator().manual_seed(seed)
    out = []
    for n in L_real:
        ids = torch.randint(1000, 30522, (n,), generator=g)
        ids[0], ids[-1] = 101, 102
        out.append((ids, torch.ones(n, dtype=torch.long), torch.randn(3, 224, 224, generator=g)))
    return out


def _oracle_logits(tr, c, e, L=512):
    from oracle import encoders as OE
    from oracle import fusion_head as OF
    sd = lambda m: {k: v.detach().float().cpu() for k, v in m.state_dict().items()}  # noqa: E731
    ids = torch.zeros(2, L, dtype=torch.long)
    mask = torch.zeros(2, L, dtype=torch.long)
    for r, (i, m, _) in enumerate((c, e)):
        ids[r, :i.numel()] = i
        mask[r, :m.numel()] = m
    px = torch.stack([c[2], e[2]])
    with torch.no_grad():
        T = OE.bert_forward(sd(tr.text_encoder), ids, mask, None, num_layers=12, num_heads=12)
        I = OE.vit_forward(sd(tr.image_encoder), px, num_layers=12, num_heads=12, patch=16)
        (a, b), (c2, d) = OF.model_forward(sd(tr.head), T[:1], I[:1], T[1:], I[1:], num_heads=8)
    return [a, b, c2, d]


@pytest.mark.parametrize("precision,tol", [("fp32", 1e-3), ("bf16", 5e-2)])
def test_predictor_graph_matches_eager_and_oracle(precision, tol):
    from mmfd.predict import PATHS, MisinformationPredictor
    from mmfd.train import build_flagship

    tr = build_flagship("cuda", precision, dropout=0.1, seed=5)
    c, e = _pair((37, 211), seed=11)
    graph = MisinformationPredictor.from_trainer(tr, use_graph=True)
    eager = MisinformationPredictor.from_trainer(tr, use_graph=False)
    got_g = [y for pair in graph.predict_logits(*c, *e) for y in pair]
    got_e = [y for pair in eager.predict_logits(*c, *e) for y in pair]
    for a, b in zip(got_g, got_e):
        assert torch.equal(a, b)
    want = _oracle_logits(tr, c, e)
    for g, w in zip(got_g, want):
        assert g.shape == w.shape == (1, 3)
        err = (g.float().cpu() - w).abs().max().item()
        assert err < tol, (precision, err)
    # a second pair through the same captured graph (static buffers are refilled, shorter text)
    c2, e2 = _pair((5, 512), seed=12)
    got2 = [y for pair in graph.predict_logits(*c2, *e2) for y in pair]
    want2 = _oracle_logits(tr, c2, e2)
    for g, w in zip(got2, want2):
        assert (g.float().cpu() - w).abs().max().item() < tol
    labels = graph.evaluate(*c2, *e2)
    assert list(labels) == list(PATHS)
    if precision == "fp32":
        for p, w in zip(PATHS, want2):
            pr = torch.softmax(w, -1)[0]
            top2 = pr.topk(2).values
            if (top2[0] - top2[1]).item() > 1e-3:  # not a near tie
                assert labels[p] == graph.idx_to_label[int(pr.argmax())]
    det = graph.evaluate(*c2, *e2, details=True)
    for p in PATHS:
        assert abs(sum(det[p]["probabilities"].values()) - 1.0) < 1e-5
        assert det[p]["label"] == labels[p]


def test_predictor_rejects_bad_pixels():
    from mmfd.predict import MisinformationPredictor
    from mmfd.train import build_flagship

    tr = build_flagship("cuda", "bf16", seed=1)
    pr = MisinformationPredictor.from_trainer(tr, use_graph=False)
    c, e = _pair((8, 8), seed=3)
    with pytest.raises(ValueError):
        pr.predict_logits(c[0], c[1], torch.zeros(3, 32, 32), *e)


def test_predictor_graph_recaptures_after_checkpoint_swap():
    """a captured graph is baked with the addresses of the bf16 weight shadows; after a
    load_state_dict of the head the graph is re-captured and equals the eager forward again."""
    from mmfd.predict import MisinformationPredictor
    from mmfd.train import build_flagship

    tr = build_flagship("cuda", "bf16", seed=6)
    c, e = _pair((40, 90), seed=13)
    graph = MisinformationPredictor.from_trainer(tr, use_graph=True)
    before = [y for pair in graph.predict_logits(*c, *e) for y in pair]
    sd = {k: v * 1.5 if k.endswith("weight") else v for k, v in tr.head.state_dict().items()}
    tr.head.load_state_dict(sd)
    after = [y for pair in graph.predict_logits(*c, *e) for y in pair]
    eager = MisinformationPredictor.from_trainer(tr, use_graph=False)
    want = [y for pair in eager.predict_logits(*c, *e) for y in pair]
    assert any(not torch.equal(a, b) for a, b in zip(before, after))
    for a, b in zip(after, want):
        assert torch.equal(a, b)
