"""TEST INFRASTRUCTURE ONLY (oracle): the full fine-tune training step of BASELINE config 3 on CPU
(bert-base + ViT-B/16 + fusion head, forward + backward + torch.optim.AdamW), composed from the
pinned restatements in oracle/encoders.py and oracle/fusion_head.py, following the reference's step
(train.py:123-188) with the encoders made trainable (BASELINE config 3 extends the reference's
frozen `no_grad` encoders, train.py:135). Used as bench.py's cpu_baseline and by parity tests.
"""
from __future__ import annotations

import torch

from . import encoders as OE
from . import fusion_head as OF


def bert_names(cfg):
    D, I, V, P, T = cfg["hidden_size"], cfg["intermediate_size"], cfg["vocab_size"], cfg["max_position_embeddings"], \
        cfg["type_vocab_size"]
    n = [("embeddings.word_embeddings.weight", [V, D]), ("embeddings.position_embeddings.weight", [P, D]),
         ("embeddings.token_type_embeddings.weight", [T, D]), ("embeddings.LayerNorm.weight", [D]),
         ("embeddings.LayerNorm.bias", [D])]
    for i in range(cfg["num_hidden_layers"]):
        p = f"encoder.layer.{i}"
        for s in ("query", "key", "value"):
            n += [(f"{p}.attention.self.{s}.weight", [D, D]), (f"{p}.attention.self.{s}.bias", [D])]
        n += [(f"{p}.attention.output.dense.weight", [D, D]), (f"{p}.attention.output.dense.bias", [D]),
              (f"{p}.attention.output.LayerNorm.weight", [D]), (f"{p}.attention.output.LayerNorm.bias", [D]),
              (f"{p}.intermediate.dense.weight", [I, D]), (f"{p}.intermediate.dense.bias", [I]),
              (f"{p}.output.dense.weight", [D, I]), (f"{p}.output.dense.bias", [D]),
              (f"{p}.output.LayerNorm.weight", [D]), (f"{p}.output.LayerNorm.bias", [D])]
    return n


def vit_names(cfg):
    D, I, C, Pz = cfg["hidden_size"], cfg["intermediate_size"], cfg["num_channels"], cfg["patch_size"]
    T = (cfg["image_size"] // Pz) ** 2 + 1
    n = [("embeddings.cls_token", [1, 1, D]), ("embeddings.position_embeddings", [1, T, D]),
         ("embeddings.patch_embeddings.projection.weight", [D, C, Pz, Pz]),
         ("embeddings.patch_embeddings.projection.bias", [D])]
    for i in range(cfg["num_hidden_layers"]):
        p = f"encoder.layer.{i}"
        for s in ("query", "key", "value"):
            n += [(f"{p}.attention.attention.{s}.weight", [D, D]), (f"{p}.attention.attention.{s}.bias", [D])]
        n += [(f"{p}.attention.output.dense.weight", [D, D]), (f"{p}.attention.output.dense.bias", [D]),
              (f"{p}.intermediate.dense.weight", [I, D]), (f"{p}.intermediate.dense.bias", [I]),
              (f"{p}.output.dense.weight", [D, I]), (f"{p}.output.dense.bias", [D]),
              (f"{p}.layernorm_before.weight", [D]), (f"{p}.layernorm_before.bias", [D]),
              (f"{p}.layernorm_after.weight", [D]), (f"{p}.layernorm_after.bias", [D])]
    n += [("layernorm.weight", [D]), ("layernorm.bias", [D])]
    return n


BERT_BASE = dict(vocab_size=30522, hidden_size=768, num_hidden_layers=12, num_attention_heads=12,
                 intermediate_size=3072, max_position_embeddings=512, type_vocab_size=2)
VIT_B16 = dict(image_size=224, patch_size=16, num_channels=3, hidden_size=768, num_hidden_layers=12,
               num_attention_heads=12, intermediate_size=3072)


class OracleTrainer:
    """CPU restatement of one full fine-tune step; params are plain tensors (name -> tensor)."""

    def __init__(self, bert_p, vit_p, head_p, bert_cfg=BERT_BASE, vit_cfg=VIT_B16, num_heads=8, lr=1e-4, drop=None):
        self.bp = {k: v.clone().float().requires_grad_(True) for k, v in bert_p.items()}
        self.vp = {k: v.clone().float().requires_grad_(True) for k, v in vit_p.items()}
        self.hp = {k: v.clone().float().requires_grad_(True) for k, v in head_p.items()}
        self.bc, self.vc, self.H = bert_cfg, vit_cfg, num_heads
        self.opt = torch.optim.AdamW(list(self.bp.values()) + list(self.vp.values()) + list(self.hp.values()), lr=lr)
        self.drop = drop

    def step(self, batch):
        self.opt.zero_grad(set_to_none=True)
        B = batch["labels"].shape[0]
        T = OE.bert_forward(self.bp, batch["input_ids"], batch["attention_mask"], None,
                            num_layers=self.bc["num_hidden_layers"], num_heads=self.bc["num_attention_heads"],
                            drop=self.drop)
        I = OE.vit_forward(self.vp, batch["pixel_values"], num_layers=self.vc["num_hidden_layers"],
                           num_heads=self.vc["num_attention_heads"], patch=self.vc["patch_size"])
        out = OF.model_forward(self.hp, T[:B], I[:B], T[B:], I[B:], num_heads=self.H, drop=self.drop)
        total, per = OF.path_loss(out, batch["labels"])
        total.backward()
        self.opt.step()
        return total.detach(), [p.detach() for p in per]


def chunked_loss_grads(bert_p, vit_p, head_p, batch, *, bert_cfg=BERT_BASE, vit_cfg=VIT_B16, num_heads=8, chunk=8,
                       drop=None, drop_head=None, progress=None):
    """The loss and parameter gradients of ONE step on a large batch (train.py:146-170 with
    trainable encoders: Σ over the 4 paths of the batch-mean cross-entropy), computed in chunks of
    `chunk` pairs so the CPU autograd graph stays small: chunk c contributes n_c / B of its own
    mean loss, so the accumulated gradients are those of the whole-batch mean.

    Dropout (layers.py:15,17,53; the encoders' hidden / attention dropout): `drop` for the text
    encoder and `drop_head` for the fusion head (default: `drop`), oracle.dropout_hash.Drop
    callbacks. Each chunk binds them to its whole-batch rows — the encoder's stacked rows [s:e] and
    [B+s:B+e], the head's rows [s:e] — so every chunk hashes the flat indices the HIP kernels hash
    for the whole batch at once, and the chunked masks are exactly the whole-batch masks.
    Returns (total, [4 path losses], {"bert."/"vit."/"head." + name: grad})."""
    import numpy as np
    bp = {k: v.clone().float().requires_grad_(True) for k, v in bert_p.items()}
    vp = {k: v.clone().float().requires_grad_(True) for k, v in vit_p.items()}
    hp = {k: v.clone().float().requires_grad_(True) for k, v in head_p.items()}
    drop_head = drop if drop_head is None else drop_head
    B = batch["labels"].shape[0]
    total = torch.zeros((), dtype=torch.float64)
    per = torch.zeros(4, dtype=torch.float64)
    for s in range(0, B, chunk):
        e = min(B, s + chunk)
        n = e - s
        ids = torch.cat([batch["input_ids"][s:e], batch["input_ids"][B + s:B + e]])
        mask = torch.cat([batch["attention_mask"][s:e], batch["attention_mask"][B + s:B + e]])
        px = torch.cat([batch["pixel_values"][s:e], batch["pixel_values"][B + s:B + e]])
        de = None if drop is None else drop.with_rows(np.concatenate([np.arange(s, e), np.arange(B + s, B + e)]))
        dh = None if drop_head is None else drop_head.with_rows(np.arange(s, e))
        T = OE.bert_forward(bp, ids, mask, None, num_layers=bert_cfg["num_hidden_layers"],
                            num_heads=bert_cfg["num_attention_heads"], drop=de)
        I = OE.vit_forward(vp, px, num_layers=vit_cfg["num_hidden_layers"],
                           num_heads=vit_cfg["num_attention_heads"], patch=vit_cfg["patch_size"])
        out = OF.model_forward(hp, T[:n], I[:n], T[n:], I[n:], num_heads=num_heads, drop=dh)
        t, pl = OF.path_loss(out, batch["labels"][s:e])
        (t * (n / B)).backward()
        total += t.detach().double() * (n / B)
        per += torch.stack([p.detach().double() for p in pl]) * (n / B)
        if progress is not None:
            progress(e, B)
    grads = {}
    for pre, d in (("bert.", bp), ("vit.", vp), ("head.", hp)):
        for k, p in d.items():
            grads[pre + k] = None if p.grad is None else p.grad.detach()
    return total, list(per), grads
