"""Cross-encoder re-ranking and the `SemanticSimilarity.search` drop-in (text
side: src/evidence/text2text_retrieval.py:10-120) on HIP kernels.

  * `BertForSequenceClassification` — HF layout (bert.*, bert.pooler.dense, classifier), the
    architecture of the reference's CrossEncoder("cross-encoder/ms-marco-MiniLM-L-6-v2")
    (text2text_retrieval.py:24): 6 post-LN BERT layers at hidden 384 / 12 heads / FFN 1536 on the
    encoder kernels of mmfd.encoders.BertModel (head dim 32), then the [CLS] pooler tanh(W h_0 + b)
    and the one-logit classifier as two small GEMMs with tanh / sigmoid epilogues. The pooler reads
    the [CLS] rows in place (a strided GEMM operand), nothing is copied.
  * `CrossEncoder.predict(pairs)` — sentence-transformers 3.3.1 semantics: (query, passage) pairs
    tokenised together (segment ids 0 / 1, padding, truncation to 512), one score per pair, the
    default activation for one label being Sigmoid.
  * `SemanticSimilarity` — the reference class: bi-encoder query embedding (fp16), util.
    semantic_search for top_k * 5 hits in the train and in the test corpus (mmfd.retrieval on the
    device-resident fp16 corpora), cross-encoder scores for every hit, each corpus' hits sorted by
    cross-score, the two lists merged and the first top_k distinct scores kept (:49-120).

Weights are random unless a state_dict is given (hub names load unchanged); tokenizers come from a
local directory (no vocabulary ships offline).
"""
from __future__ import annotations

import os

import numpy as np
import torch
import torch.nn as nn

from . import blocks as Bk
from . import kernels as K
from .encoders import BertConfig, BertModel
from .retrieval import CorpusIndex, semantic_search


def minilm_l6_config(**kw):
    """cross-encoder/ms-marco-MiniLM-L-6-v2 (BertForSequenceClassification, num_labels 1)"""
    return BertConfig(**{**dict(vocab_size=30522, hidden_size=384, num_hidden_layers=6, num_attention_heads=12,
                                intermediate_size=1536, max_position_embeddings=512, type_vocab_size=2), **kw})


class BertForSequenceClassification(Bk.CachedWeights, nn.Module):
    """HF BertForSequenceClassification (inference): forward -> logits [B, num_labels] fp32."""

    def __init__(self, config: BertConfig | None = None, num_labels=1):
        super().__init__()
        c = config or minilm_l6_config()
        self.config, self.num_labels = c, num_labels
        self.bert = BertModel(c)
        self.bert.pooler = nn.Module()
        self.bert.pooler.dense = nn.Linear(c.hidden_size, c.hidden_size)
        self.classifier = nn.Linear(c.hidden_size, num_labels)
        for m in (self.bert.pooler.dense, self.classifier):
            nn.init.normal_(m.weight, 0.0, 0.02)
            nn.init.zeros_(m.bias)
        self.compute_dtype = torch.float32
        self.eval()

    def set_precision(self, precision):
        self.compute_dtype = {"fp32": torch.float32, "bf16": torch.bfloat16}[precision]
        self.bert.set_precision(precision)
        return self

    @torch.no_grad()
    def forward(self, input_ids, attention_mask=None, token_type_ids=None, activation=None):
        """logits (activation None) or activation(logits) ('sigmoid'), fp32 [B, num_labels]"""
        h = self.bert(input_ids=input_ids, attention_mask=attention_mask,
                      token_type_ids=token_type_ids).last_hidden_state          # [B, L, D]
        P = {n: p.detach() for n, p in self.named_parameters()}
        sc = Bk.StepCtx(P, self.compute_dtype, shadows=Bk.shadow_store(self))
        cls = h[:, 0]                                                          # [B, D] view, ld = L * D
        pooled = K.gemm(cls, sc.w("bert.pooler.dense"), bias=P["bert.pooler.dense.bias"], act=K.ACT_TANH)
        act = K.ACT_SIGMOID if activation == "sigmoid" else K.ACT_NONE
        if activation not in (None, "sigmoid"):
            raise ValueError("activation must be None or 'sigmoid'")
        return K.gemm(pooled, sc.w("classifier"), bias=P["classifier.bias"], act=act, out_dtype=torch.float32)


class CrossEncoder:
    """sentence_transformers.CrossEncoder (predict) on a HIP BertForSequenceClassification."""

    def __init__(self, model: BertForSequenceClassification | None = None, tokenizer=None, max_length=512,
                 device="cuda", precision="fp32", default_activation="sigmoid", state_dict=None):
        self.model = model if model is not None else BertForSequenceClassification()
        if state_dict is not None:  # (the tokenizer-side position_ids buffer of HF checkpoints is benign)
            Bk.load_state_dict_checked(self.model, state_dict)
        self.model = self.model.to(device).eval().set_precision(precision)
        self.tokenizer, self.max_length, self.device = tokenizer, max_length, torch.device(device)
        self.default_activation = default_activation if self.model.num_labels == 1 else None

    def predict_ids(self, input_ids, attention_mask, token_type_ids, batch_size=256, activation="default"):
        """scores fp32 [N] (num_labels 1) or [N, num_labels] of pre-tokenised pairs"""
        act = self.default_activation if activation == "default" else activation
        outs = []
        for i in range(0, input_ids.shape[0], batch_size):
            sl = slice(i, i + batch_size)
            outs.append(self.model(input_ids[sl].to(self.device), attention_mask[sl].to(self.device),
                                   token_type_ids[sl].to(self.device), activation=act))
        y = torch.cat(outs) if len(outs) > 1 else outs[0]
        return y[:, 0] if self.model.num_labels == 1 else y

    def predict(self, sentences, batch_size=32, activation="default", convert_to_numpy=True):
        """CrossEncoder.predict([[query, passage], ...]) -> one score per pair"""
        if self.tokenizer is None:
            raise RuntimeError("CrossEncoder.predict needs a tokenizer (no vocabulary ships offline)")
        if len(sentences) == 0:
            return np.zeros(0, np.float32) if convert_to_numpy else torch.zeros(0)
        a, b = [s[0] for s in sentences], [s[1] for s in sentences]
        enc = self.tokenizer(a, b, padding=True, truncation="longest_first", return_tensors="pt",
                             max_length=self.max_length)
        tts = enc.get("token_type_ids")
        if tts is None:
            tts = torch.zeros_like(enc["input_ids"])
        s = self.predict_ids(enc["input_ids"], enc["attention_mask"], tts, batch_size=max(batch_size, 256),
                             activation=activation).float().cpu()
        return s.numpy() if convert_to_numpy else s


class SemanticSimilarity:
    """text2text_retrieval.py:10-120 on HIP: bi-encoder search over the train and test embedding
    files (`{split}_embeddings.h5|npz` from mmfd.evidence.TextCorpus), cross-encoder re-rank,
    merge and distinct-score filter."""

    def __init__(self, train_embeddings_file, test_embeddings_file, train_csv_path=None, test_csv_path=None,
                 train_df=None, test_df=None, bi_encoder=None, cross_encoder=None, device="cuda"):
        import pandas as pd
        from .evidence import SentenceEncoder
        self.bi_encoder = bi_encoder if bi_encoder is not None else SentenceEncoder(device=device, max_seq_length=512)
        self.cross_encoder = cross_encoder if cross_encoder is not None else CrossEncoder(device=device)
        self.train_embeddings, self.train_ids = self._load_embeddings(train_embeddings_file)
        self.test_embeddings, self.test_ids = self._load_embeddings(test_embeddings_file)
        self.train_csv = train_df if train_df is not None else pd.read_csv(train_csv_path)
        self.test_csv = test_df if test_df is not None else pd.read_csv(test_csv_path)
        # the fp16 corpora stay resident in HBM for every search
        self._train_index = CorpusIndex(self.train_embeddings, device=device, mode="normalized", round_f16=True)
        self._test_index = CorpusIndex(self.test_embeddings, device=device, mode="normalized", round_f16=True)
        self.device = device

    @staticmethod
    def _load_embeddings(path):
        """(fp16 tensor [N, D], ids as str) — text2text_retrieval.py:39-47 (ids decoded as :99-104)"""
        from .evidence import TextCorpus
        emb, ids = TextCorpus.read(path)
        return torch.as_tensor(np.asarray(emb), dtype=torch.float16), [i.decode("utf-8") if isinstance(i, bytes) else
                                                                         str(i) for i in ids]

    def _rerank(self, query, hits, csv, top_k):
        cross_inp = [[query, csv["evidence_enriched"][h["corpus_id"]]] for h in hits]
        scores = self.cross_encoder.predict(cross_inp)
        for h, s in zip(hits, scores):
            h["cross-score"] = float(s)
        return sorted(hits, key=lambda x: x.get("cross-score"), reverse=True)[: top_k * 5]

    def search(self, query, top_k):
        q = self.bi_encoder.encode([query]).to(dtype=torch.float16)        # :52-54
        qd = q.to(self.device)
        hits_train = semantic_search(qd, self._train_index, top_k=top_k * 5)[0]   # :56-59
        hits_test = semantic_search(qd, self._test_index, top_k=top_k * 5)[0]     # :61-64
        hits_train = self._rerank(query, hits_train, self.train_csv, top_k)        # :68-94
        hits_test = self._rerank(query, hits_test, self.test_csv, top_k)
        results = [(self.train_ids[h["corpus_id"]], h.get("cross-score")) for h in hits_train] + \
                  [(self.test_ids[h["corpus_id"]], h.get("cross-score")) for h in hits_test]  # :96-103
        seen, out = set(), []
        for id_, score in sorted(results, key=lambda x: x[1], reverse=True):    # :105-118
            if score not in seen:
                seen.add(score)
                out.append((id_, score))
            if len(out) == top_k:
                break
        return out
