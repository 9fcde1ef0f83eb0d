"""One small training step of the flagship path (BERT + ViT + fusion head + AdamW) on the HIP
device, checked against the CPU oracle (oracle/train_step.py) — the body of
__graft_entry__.smoke() and of tests/test_trainer_gpu.py.

Test infrastructure: the oracle is only the checker here; the step under test runs through
libmmfd_hip.so (FusionTrainer -> HIP kernels) and fails loudly if the library is missing.
"""
from __future__ import annotations

import torch

import mmfd
from mmfd import kernels as K
from mmfd.encoders import BertConfig, BertModel, ViTConfig, ViTModel
from mmfd.model import MisinformationDetectionModel
from mmfd.train import FusionTrainer
from oracle.dropout_hash import make_drop
from oracle.train_step import OracleTrainer

TINY = dict(D=64, layers=2, heads=4, inter=128, vocab=120, seq=16, img=32, patch=8, embed=32, head_heads=4,
            hidden=16)
# BASELINE config 3 at full size: bert-base-uncased + ViT-B/16 + the fusion head (768/768, E=256, H=8)
FULL = dict(D=768, layers=12, heads=12, inter=3072, vocab=30522, seq=128, img=224, patch=16, embed=256, head_heads=8,
            hidden=64)


def tiny_batch(B, cfg=TINY, seed=0, ragged=True):
    g = torch.Generator().manual_seed(seed)
    L, V = cfg["seq"], cfg["vocab"]
    ids = torch.randint(3, V, (2 * B, L), generator=g)
    n = torch.randint(4, L + 1, (2 * B,), generator=g) if ragged else torch.full((2 * B,), L)
    mask = (torch.arange(L)[None] < n[:, None]).long()
    ids = ids * mask
    labels = torch.randint(0, 3, (B, 4), generator=g)
    px = torch.randn(2 * B, 3, cfg["img"], cfg["img"], generator=g)
    return {"input_ids": ids, "attention_mask": mask, "pixel_values": px, "labels": labels}


def build_modules(dropout=0.1, cfg=TINY, seed=5):
    """(text, image, head) mmfd modules on the CPU from `seed`, and their initial state_dicts
    (the weights the oracle starts from; tests/golden/make_config3_bs256.py uses the same recipe)."""
    torch.manual_seed(seed)
    bc = BertConfig(vocab_size=cfg["vocab"], hidden_size=cfg["D"], num_hidden_layers=cfg["layers"],
                    num_attention_heads=cfg["heads"], intermediate_size=cfg["inter"],
                    max_position_embeddings=max(64, cfg["seq"]),
                    hidden_dropout_prob=dropout, attention_probs_dropout_prob=dropout)
    vc = ViTConfig(image_size=cfg["img"], patch_size=cfg["patch"], hidden_size=cfg["D"],
                   num_hidden_layers=cfg["layers"], num_attention_heads=cfg["heads"], intermediate_size=cfg["inter"])
    text, image = BertModel(bc), ViTModel(vc)
    head = MisinformationDetectionModel(text_input_dim=cfg["D"], image_input_dim=cfg["D"], embed_dim=cfg["embed"],
                                        num_heads=cfg["head_heads"], dropout=dropout, hidden_dim=cfg["hidden"])
    states = [{k: v.detach().clone() for k, v in m.state_dict().items()} for m in (text, image, head)]
    return text, image, head, states


def oracle_cfgs(cfg):
    bcfg = dict(hidden_size=cfg["D"], num_hidden_layers=cfg["layers"], num_attention_heads=cfg["heads"])
    vcfg = dict(patch_size=cfg["patch"], num_hidden_layers=cfg["layers"], num_attention_heads=cfg["heads"])
    return bcfg, vcfg


def build_pair(precision="fp32", dropout=0.1, cfg=TINY, seed=5, lr=1e-3, with_oracle=True):
    """(HIP FusionTrainer on cuda:0, OracleTrainer on CPU) with identical initial weights and dropout masks."""
    text, image, head, states = build_modules(dropout, cfg, seed)
    dev = torch.device("cuda", 0)
    text, image, head = text.to(dev), image.to(dev), head.to(dev)
    text.manual_seed(99)
    head.manual_seed(99)  # same seed: every dropout site has its own salt
    tr = FusionTrainer(text, image, head, lr=lr, precision=precision)
    if not with_oracle:
        return tr, states
    bcfg, vcfg = oracle_cfgs(cfg)
    ref = OracleTrainer(*states, bert_cfg=bcfg, vit_cfg=vcfg, num_heads=cfg["head_heads"], lr=lr,
                        drop=make_drop(99, dropout) if dropout > 0 else None)
    return tr, ref


def _named(tr):
    out = {}
    for pre, m in (("bert.", tr.text_encoder), ("vit.", tr.image_encoder), ("head.", tr.head)):
        for k, p in m.named_parameters():
            out[pre + k] = p
    return out


def _named_ref(ref):
    out = {}
    for pre, d in (("bert.", ref.bp), ("vit.", ref.vp), ("head.", ref.hp)):
        for k, p in d.items():
            out[pre + k] = p
    return out


def compare_step(tr, ref, batch, loss_tol, grad_rtol, norm_rtol=None, report=None):
    """One step on each; returns (max loss err, worst grad error relative to that tensor's max
    |grad|). With `norm_rtol`, every gradient must also satisfy ||g - r||_2 / ||r||_2 <= norm_rtol;
    `report` (a list) receives (name, max-relative, norm-relative) per tensor."""
    dev = torch.device("cuda", 0)
    tr.text_encoder.manual_seed(99)  # the oracle's make_drop(99, p) masks, every step
    tr.head.manual_seed(99)
    loss = tr.step({k: v.to(dev) for k, v in batch.items()})
    torch.cuda.synchronize()
    rl, rper = ref.step(batch)
    got = loss.double().cpu()
    want = torch.stack([rl] + list(rper)).double()
    lerr = (got - want).abs().max().item()
    assert lerr <= loss_tol, f"loss mismatch {got.tolist()} vs {want.tolist()}"
    mine, theirs = _named(tr), _named_ref(ref)
    assert mine.keys() == theirs.keys()
    worst = 0.0
    # gradients that are zero in exact arithmetic (e.g. key biases: softmax is shift invariant)
    # are fp32 noise in both; judge every tensor against at least 1e-3 of the largest gradient
    floor = 1e-3 * max(r.grad.abs().max().item() for r in theirs.values() if r.grad is not None)
    nfloor = 1e-3 * max(r.grad.norm().item() for r in theirs.values() if r.grad is not None)
    fails = []
    for k, p in mine.items():
        g, r = p.grad, theirs[k].grad
        if r is None:
            assert g is None or g.abs().max().item() == 0.0, k
            continue
        assert g is not None, f"missing grad {k}"
        d = g.double().cpu() - r.double()
        e = d.abs().max().item() / max(r.abs().max().item(), floor)
        en = d.norm().item() / max(r.double().norm().item(), nfloor)
        if report is not None:
            report.append((k, e, en))
        if e > grad_rtol or (norm_rtol is not None and en > norm_rtol):
            fails.append(f"grad {k}: max-rel {e:.2e} (bound {grad_rtol:.1e}), norm-rel {en:.2e} (bound {norm_rtol})")
        worst = max(worst, e)
    assert not fails, "; ".join(fails[:8])
    return lerr, worst


def run_smoke():
    if not torch.cuda.is_available():
        raise RuntimeError("smoke() needs a HIP device (cuda:0)")
    K.load()  # loud failure if libmmfd_hip.so is missing
    tr, ref = build_pair("fp32", dropout=0.1)
    batch = tiny_batch(2, seed=11)
    l1, g1 = compare_step(tr, ref, batch, loss_tol=1e-3, grad_rtol=2e-3)
    l2, g2 = compare_step(tr, ref, tiny_batch(2, seed=12), loss_tol=1e-3, grad_rtol=2e-3)
    print(f"smoke ok (mmfd {mmfd.__version__}, {K.LIB_PATH}): fp32 train step vs oracle, "
          f"loss err {max(l1, l2):.2e}, worst rel grad err {max(g1, g2):.2e}", flush=True)


if __name__ == "__main__":
    run_smoke()
