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
