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
    from mmfd.predict import PATHS, PairPredictor
    from mmfd.train import build_flagship

    tr = build_flagship("cuda", precision, dropout=0.1, seed=5)
    c, e = _pair((37, 211), seed=11)
    graph = PairPredictor.from_trainer(tr, use_graph=True)
    eager = PairPredictor.from_trainer(tr, use_graph=False)
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
    from mmfd.predict import PairPredictor
    from mmfd.train import build_flagship

    tr = build_flagship("cuda", "bf16", seed=1)
    pr = PairPredictor.from_trainer(tr, use_graph=False)
    c, e = _pair((8, 8), seed=3)
    with pytest.raises(ValueError):
        pr.predict_logits(c[0], c[1], torch.zeros(3, 32, 32), *e)


def test_predictor_graph_recaptures_after_checkpoint_swap():
    """a captured graph is baked with the addresses of the bf16 weight shadows; after a
    load_state_dict of the head the graph is re-captured and equals the eager forward again."""
    from mmfd.predict import PairPredictor
    from mmfd.train import build_flagship

    tr = build_flagship("cuda", "bf16", seed=6)
    c, e = _pair((40, 90), seed=13)
    graph = PairPredictor.from_trainer(tr, use_graph=True)
    before = [y for pair in graph.predict_logits(*c, *e) for y in pair]
    sd = {k: v * 1.5 if k.endswith("weight") else v for k, v in tr.head.state_dict().items()}
    tr.head.load_state_dict(sd)
    after = [y for pair in graph.predict_logits(*c, *e) for y in pair]
    eager = PairPredictor.from_trainer(tr, use_graph=False)
    want = [y for pair in eager.predict_logits(*c, *e) for y in pair]
    assert any(not torch.equal(a, b) for a, b in zip(before, after))
    for a, b in zip(after, want):
        assert torch.equal(a, b)


# ---- the evaluate.py drop-in: checkpoint path, raw strings, image files --------------------------
def _oracle_pair(pred, c_text, c_img, e_text, e_img):
    """the reference computation of evaluate.py:95-165 on the CPU oracle: tokenise to 512 with
    padding, DeBERTa-v3 (oracle/deberta.py) on each text, Resize((256, 256)) + ImageNet Normalize
    (oracle/preprocess.py) and Swinv2 (oracle/swinv2.py) on each readable image, the fusion head
    (oracle/fusion_head.py) with None for a missing image"""
    from PIL import Image
    from mmfd.preprocess import MODES
    from oracle import fusion_head as OF
    from oracle.deberta import deberta_forward
    from oracle.preprocess import preprocess
    from oracle.swinv2 import swinv2_forward
    sd = lambda m: {k: v.detach().float().cpu() for k, v in m.state_dict().items()}  # noqa: E731
    te = pred.text_encoder
    P = sd(te)
    cfg = MODES["evaluate"]
    with torch.no_grad():
        T = []
        for text in (c_text, e_text):
            enc = pred.tokenizer(text, truncation=True, padding="max_length", max_length=512, return_tensors="pt")
            T.append(deberta_forward(P, enc["input_ids"], enc["attention_mask"], num_layers=te.config.num_hidden_layers,
                                     num_heads=te.config.num_attention_heads, eps=te.config.layer_norm_eps))
        I = []
        for path in (c_img, e_img):
            try:
                img = Image.open(path)
            except Exception:
                I.append(None)
                continue
            px = torch.from_numpy(preprocess(img, cfg["resize"], cfg["crop"], cfg["mean"], cfg["std"]))[None]
            I.append(swinv2_forward(sd(pred.image_encoder), px)[0])
        (a, b), (c, d) = OF.model_forward(sd(pred.model), T[0], I[0], T[1], I[1], num_heads=8)
    return [a, b, c, d]


@pytest.fixture
def predictor_files(tmp_path):
    import numpy as np
    from PIL import Image
    from mmfd.model import MisinformationDetectionModel
    torch.manual_seed(17)
    head = MisinformationDetectionModel(text_input_dim=384, image_input_dim=1024)  # the reference's defaults
    ck = tmp_path / "model.pt"
    torch.save({"model_state_dict": head.state_dict(), "epoch": 1}, ck)  # train.py's checkpoint layout
    rng = np.random.default_rng(5)
    paths = []
    for name, (h, w) in (("claim.png", (300, 410)), ("evidence.jpg", (257, 256))):
        p = tmp_path / name
        Image.fromarray(rng.integers(0, 256, (h, w, 3), dtype=np.uint8)).save(p)
        paths.append(str(p))
    return str(ck), paths, tmp_path


def test_misinformation_predictor_reference_api(predictor_files):
    """evaluate.py's contract end to end: MisinformationPredictor(model_path,
    device, ..., text_input_dim=384, image_input_dim=1024, text_encoder="microsoft/deberta-v3-xsmall")
    loads the checkpoint's model_state_dict, builds DeBERTa-v3-xsmall + Swinv2-base (seeded random
    weights: no hub offline), and evaluate(claim_text, claim_image_path, evidence_text,
    evidence_image_path) returns the per-path labels of the oracle's logits (fp32 logits within
    north_star's 1e-3 at L = 512 through the captured graph). An unreadable evidence image makes
    that modality None: text_image / image_image come back None and the other two paths match the
    oracle run with E_i = None (evaluate.py:141-156); an evaluation failure returns None."""
    import random
    from mmfd.predict import PATHS, MisinformationPredictor
    from tests.toy_tokenizer import WORDS, toy_tokenizer
    ck, (c_img, e_img), tmp = predictor_files
    pred = MisinformationPredictor(ck, device="cuda", tokenizer=toy_tokenizer(), seed=3)
    rnd = random.Random(7)
    c_text = " ".join(rnd.choice(WORDS) for _ in range(40))
    e_text = " ".join(rnd.choice(WORDS) for _ in range(700))  # longer than 512 tokens: truncated
    got = [y for pair in pred.predict_logits(c_text, c_img, e_text, e_img) for y in pair]
    want = _oracle_pair(pred, c_text, c_img, e_text, e_img)
    for g, w in zip(got, want):
        assert g.shape == w.shape == (1, 3)
        assert (g.float().cpu() - w).abs().max().item() < 1e-3
    labels = pred.evaluate(c_text, c_img, e_text, e_img)
    assert list(labels) == list(PATHS)
    for p, w in zip(PATHS, want):
        pr = torch.softmax(w, -1)[0]
        if (pr.topk(2).values[0] - pr.topk(2).values[1]).item() > 1e-3:
            assert labels[p] == pred.idx_to_label[int(pr.argmax())], p
    # a missing evidence image: that modality is None
    missing = str(tmp / "no_such_image.jpg")
    got = [y for pair in pred.predict_logits(c_text, c_img, e_text, missing) for y in pair]
    want = _oracle_pair(pred, c_text, c_img, e_text, missing)
    assert got[1] is None and got[3] is None and want[1] is None and want[3] is None
    for g, w in ((got[0], want[0]), (got[2], want[2])):
        assert (g.float().cpu() - w).abs().max().item() < 1e-3
    labels = pred.evaluate(c_text, c_img, e_text, missing)
    assert labels["text_image"] is None and labels["image_image"] is None
    assert labels["text_text"] in pred.idx_to_label.values() and labels["image_text"] in pred.idx_to_label.values()
    # both images missing: only the text-text path
    labels = pred.evaluate(c_text, missing, e_text, missing)
    assert labels["text_text"] is not None and all(labels[p] is None for p in PATHS[1:])
    # a failure of the evaluation itself (here: a non-string text) is logged and returns None
    assert pred.evaluate(None, c_img, e_text, e_img) is None
