"""Cross-encoder re-ranking and SemanticSimilarity.search (text2text_retrieval.py:
10-120) on the HIP path.

* BertForSequenceClassification (the ms-marco-MiniLM-L-6-v2 cross-encoder architecture) vs the
  transformers fixture (tests/golden/cross_encoder_small.npz): fp32 logits and sigmoid scores
  <= 1e-4, bf16 <= 2e-2 (sentence-transformers itself is absent: the CrossEncoder wrapper's
  pairing / segment ids / default Sigmoid are restated, parity of those pinned by the oracle only);
* the full MiniLM-L6 shape (hidden 384, 12 heads of 32, 6 layers) at up to 512 tokens vs the CPU
  oracle with recipe weights: fp32 <= 1e-4 on the sigmoid scores, <= 1e-3 on the logits;
* SemanticSimilarity.search end to end (toy vocabulary, small random MPNet bi-encoder and
  cross-encoder, fp16 train / test corpora on disk) vs the oracle's restatement of :49-120 — the
  same top_k * 5 candidates per corpus, the same cross-scores (<= 1e-5) and the same merged,
  distinct-score result; a passage planted twice in the train corpus is returned once.
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle import encoders as OE
from oracle.fusion_head import init_params_like_reference
from oracle.retrieval import cosine_normalized, ranked
from tests.toy_tokenizer import sentence, toy_tokenizer

pytestmark = pytest.mark.gpu
DEV = "cuda"
G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _fixture_model(precision):
    from mmfd.encoders import BertConfig
    from mmfd.rerank import BertForSequenceClassification
    z = np.load(os.path.join(G, "cross_encoder_small.npz"))
    cfg = json.loads(str(z["config"]))
    cfg.pop("num_labels")
    m = BertForSequenceClassification(BertConfig(**cfg), num_labels=1)
    sd = {k[len("param/"):]: torch.from_numpy(z[k]) for k in z.files if k.startswith("param/")}
    sd.pop("bert.embeddings.position_ids", None)
    m.load_state_dict(sd)
    return z, m.to(DEV).set_precision(precision)


@pytest.mark.parametrize("precision,tol", [("fp32", 1e-4), ("bf16", 2e-2)])
def test_cross_encoder_matches_transformers_fixture(precision, tol):
    z, m = _fixture_model(precision)
    args = [torch.from_numpy(z[k]).to(DEV) for k in ("input_ids", "attention_mask", "token_type_ids")]
    logits = m(*args)
    scores = m(*args, activation="sigmoid")
    torch.cuda.synchronize()
    assert logits.shape == (4, 1) and logits.dtype == torch.float32
    assert (logits.cpu() - torch.from_numpy(z["logits"])).abs().max().item() <= tol
    assert (scores.cpu() - torch.from_numpy(z["scores"])).abs().max().item() <= tol


def test_minilm_l6_full_shape_matches_oracle():
    from mmfd.rerank import BertForSequenceClassification, CrossEncoder, minilm_l6_config
    m = BertForSequenceClassification(minilm_l6_config())
    names = [(k, list(v.shape)) for k, v in m.state_dict().items()]
    P = init_params_like_reference(names, 29)
    m.load_state_dict(P)
    ce = CrossEncoder(m, device=DEV, precision="fp32")
    g = torch.Generator().manual_seed(3)
    B, L = 5, 512
    lens = torch.tensor([512, 300, 77, 12, 450])
    qlen = torch.tensor([20, 9, 30, 4, 64])
    pos = torch.arange(L)[None]
    mask = (pos < lens[:, None]).long()
    tts = ((pos >= qlen[:, None]) & (pos < lens[:, None])).long()
    ids = torch.randint(1000, 30522, (B, L), generator=g) * mask
    got = ce.predict_ids(ids, mask, tts).cpu()
    got_logits = ce.predict_ids(ids, mask, tts, activation=None).cpu()
    with torch.no_grad():
        want = OE.cross_encoder_forward(P, ids, mask, tts, num_layers=6, num_heads=12)[:, 0]
        want_logits = OE.cross_encoder_forward(P, ids, mask, tts, num_layers=6, num_heads=12, activation=None)[:, 0]
    assert (got - want).abs().max().item() <= 1e-4
    assert (got_logits - want_logits).abs().max().item() <= 1e-3


def _small_mpnet(seed):
    from mmfd.encoders import MPNetConfig, MPNetModel
    torch.manual_seed(seed)
    return MPNetModel(MPNetConfig(vocab_size=100, hidden_size=64, num_hidden_layers=2, num_attention_heads=2,
                                  intermediate_size=128, max_position_embeddings=80))


def test_semantic_similarity_search_matches_oracle(tmp_path):
    import pandas as pd
    from mmfd.encoders import BertConfig
    from mmfd.evidence import SentenceEncoder
    from mmfd.rerank import BertForSequenceClassification, CrossEncoder, SemanticSimilarity

    rng = np.random.default_rng(5)
    tok = toy_tokenizer()
    dfs = {}
    # corpora no larger than top_k * 5: every entry is a bi-encoder candidate, so the comparison is
    # not decided by fp16 score ties at the candidate boundary (util.semantic_search itself is
    # pinned in tests/test_retrieval_gpu.py)
    for split, n in (("train", 20), ("test", 14)):
        texts = [sentence(rng) for _ in range(n)]
        if split == "train":
            texts[17] = texts[3]  # the same passage twice: one cross-score, kept once
        dfs[split] = pd.DataFrame({"id": list(range(100, 100 + n)), "evidence_enriched": texts})
    bi = SentenceEncoder(_small_mpnet(7), device=DEV, precision="fp32", tokenizer=tok, max_seq_length=64)
    torch.manual_seed(8)
    ce_model = BertForSequenceClassification(BertConfig(vocab_size=100, hidden_size=64, num_hidden_layers=2,
                                                        num_attention_heads=2, intermediate_size=128,
                                                        max_position_embeddings=80))
    with torch.no_grad():  # spread the random scores (hub-scale init gives logits within 1e-5 of 0)
        torch.nn.init.normal_(ce_model.bert.pooler.dense.weight, 0.0, 0.3)
        torch.nn.init.normal_(ce_model.classifier.weight, 0.0, 1.0)
    ce = CrossEncoder(ce_model, tokenizer=tok, max_length=80, device=DEV, precision="fp32")
    files = {}
    for split, df in dfs.items():  # the corpus files exactly as TextCorpus writes them (fp16 + ids)
        emb = bi.encode(df["evidence_enriched"].tolist()).numpy().astype(np.float16)
        files[split] = str(tmp_path / f"{split}_embeddings.npz")
        np.savez(files[split], embeddings=emb, ids=np.array([f"{split}_{i}" for i in df["id"]]))
    sim = SemanticSimilarity(files["train"], files["test"], train_df=dfs["train"], test_df=dfs["test"],
                             bi_encoder=bi, cross_encoder=ce, device=DEV)
    Pce = {k: v.detach().cpu() for k, v in ce.model.state_dict().items()}
    query = sentence(rng, 4, 10)
    top_k = 4
    got = sim.search(query, top_k)

    # ---- oracle restatement of text2text_retrieval.py:49-120 -----------------------------------
    q16 = bi.encode(query).half().float().numpy()[None]
    merged = []
    for split in ("train", "test"):
        emb = np.load(files[split])["embeddings"].astype(np.float32)
        sc = cosine_normalized(q16, emb)[0].astype(np.float16).astype(np.float64)  # fp16 scores
        hits = [int(i) for i in ranked(sc)[: top_k * 5]]
        enc = tok([query] * len(hits), [dfs[split]["evidence_enriched"][h] for h in hits], padding=True,
                  truncation="longest_first", return_tensors="pt", max_length=80)
        with torch.no_grad():
            cs = OE.cross_encoder_forward(Pce, enc["input_ids"], enc["attention_mask"], enc["token_type_ids"],
                                          num_layers=2, num_heads=2)[:, 0].double().numpy()
        order = sorted(range(len(hits)), key=lambda j: cs[j], reverse=True)[: top_k * 5]
        merged += [(f"{split}_{dfs[split]['id'][hits[j]]}", float(cs[j])) for j in order]
    want, seen = [], []
    for id_, s in sorted(merged, key=lambda x: x[1], reverse=True):
        if not any(abs(s - t) <= 1e-6 for t in seen):
            seen.append(s)
            want.append((id_, s))
        if len(want) == top_k:
            break
    assert [g[0] for g in got] == [w[0] for w in want], (got, want)
    for (_, a), (_, b) in zip(got, want):
        assert abs(a - b) <= 1e-5
    dup = {f"train_{dfs['train']['id'][3]}", f"train_{dfs['train']['id'][17]}"}
    assert len(dup & {g[0] for g in sim.search(dfs["train"]["evidence_enriched"][3], 10)}) <= 1
