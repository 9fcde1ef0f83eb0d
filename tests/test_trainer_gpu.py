"""Whole training step (BERT + ViT + fusion head + AdamW, FusionTrainer) on the HIP path vs the
CPU oracle's step (oracle/train_step.py, restating train.py:123-188 with trainable encoders).

Tolerances: fp32 — losses 1e-3 abs (north_star), every parameter gradient 2e-3 relative to that
tensor's max |grad|, over two consecutive steps (the second starts from AdamW-updated weights);
bf16 — losses 5e-2 abs, gradients 0.1 relative (bf16 operands, fp32 accumulation/master weights).
"""
import pytest
import torch

from tests.smoke_impl import TINY, build_pair, compare_step, tiny_batch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("gelu_deriv", [True, False])
@pytest.mark.parametrize("dropout", [0.0, 0.1])
def test_train_step_fp32_matches_oracle(dropout, gelu_deriv, monkeypatch):
    """(gelu_deriv: the FFN forward saves gelu'(pre-activation) — MMFD_ACT_GELU_D — or the
    pre-activation, blocks.GELU_DERIV)"""
    from mmfd import blocks as Bk
    monkeypatch.setattr(Bk, "GELU_DERIV", gelu_deriv)
    tr, ref = build_pair("fp32", dropout=dropout)
    for s in (1, 2):
        compare_step(tr, ref, tiny_batch(3, seed=s), loss_tol=1e-3, grad_rtol=2e-3)


def test_train_step_fp32_wider_matches_oracle():
    cfg = dict(TINY, D=128, heads=2, inter=256, seq=40, img=48, patch=16, embed=64, head_heads=8)
    tr, ref = build_pair("fp32", dropout=0.1, cfg=cfg)
    compare_step(tr, ref, tiny_batch(2, cfg=cfg, seed=3), loss_tol=1e-3, grad_rtol=2e-3)


@pytest.mark.parametrize("gelu_deriv", [True, False])
def test_train_step_bf16_close_to_oracle(gelu_deriv, monkeypatch):
    from mmfd import blocks as Bk
    monkeypatch.setattr(Bk, "GELU_DERIV", gelu_deriv)
    tr, ref = build_pair("bf16", dropout=0.0)
    compare_step(tr, ref, tiny_batch(3, seed=4), loss_tol=5e-2, grad_rtol=0.1)


def test_frozen_encoders_only_head_updates():
    tr, _ = build_pair("fp32", dropout=0.0)
    from mmfd.train import FusionTrainer

    ft = FusionTrainer(tr.text_encoder, tr.image_encoder, tr.head, freeze_encoders=True, precision="fp32")
    before = [p.detach().clone() for p in tr.text_encoder.parameters()]
    hb = [p.detach().clone() for p in tr.head.parameters()]
    ft.step({k: v.cuda() for k, v in tiny_batch(2, seed=9).items()})
    torch.cuda.synchronize()
    assert all(torch.equal(a, b) for a, b in zip(before, tr.text_encoder.parameters()))
    assert any(not torch.equal(a, b) for a, b in zip(hb, tr.head.parameters()))


@pytest.mark.parametrize("precision,tol", [("fp32", 1e-3), ("bf16", 5e-2)])
def test_config2_full_size_forward_logits(precision, tol):
    """BASELINE config 2 at full size: bert-base-uncased + ViT-B/16 + the fusion head (768/768,
    E=256, H=8), eval-mode forward of claim/evidence pairs (ragged text masks), logits vs the CPU
    oracle (oracle/encoders.py + oracle/fusion_head.py). Tolerance: north_star's 1e-3 abs in fp32;
    5e-2 abs in bf16 (SURVEY 7 "Hard parts": bf16 moves logits by up to 1.8e-2)."""
    from mmfd.train import build_flagship
    from oracle import encoders as OE
    from oracle import fusion_head as OF
    from mmfd.dataset import synthetic_batch

    tr = build_flagship("cuda", precision, dropout=0.1, seed=3)
    B = 2
    batch = synthetic_batch(B, seed=17, device="cpu", ragged=True)
    out = tr.predict({k: v.cuda() for k, v in batch.items()})
    torch.cuda.synchronize()
    sd = lambda m: {k: v.detach().float().cpu() for k, v in m.state_dict().items()}  # noqa: E731
    bp, vp, hp = sd(tr.text_encoder), sd(tr.image_encoder), sd(tr.head)
    with torch.no_grad():
        T = OE.bert_forward(bp, batch["input_ids"], batch["attention_mask"], None, num_layers=12, num_heads=12)
        I = OE.vit_forward(vp, batch["pixel_values"], num_layers=12, num_heads=12, patch=16)
        ref = OF.model_forward(hp, T[:B], I[:B], T[B:], I[B:], num_heads=8)
    got = [y for pair in out for y in pair]
    want = [y for pair in ref for y in pair]
    for g, w in zip(got, want):
        assert g.shape == w.shape
        err = (g.float().cpu() - w).abs().max().item()
        assert err < tol, (precision, err)


def test_bf16_weight_shadows_follow_adamw_and_external_updates():
    """bf16 steps read persistent bf16 copies of the master weights that mmfd AdamW refreshes in
    its own launch: after several steps every registered copy equals bf16(master) exactly, and an
    in-place update made outside AdamW (version bump) forces a re-cast on the next forward."""
    from mmfd import blocks as Bk
    from mmfd import kernels as K
    tr, _ = build_pair("bf16", dropout=0.1)
    for s in range(3):
        tr.step({k: v.cuda() for k, v in tiny_batch(2, seed=30 + s).items()})
    torch.cuda.synchronize()
    named = {}
    for m in (tr.text_encoder, tr.image_encoder, tr.head):
        named.update({p.data_ptr(): p for p in m.parameters()})
    checked = 0
    for m in (tr.text_encoder, tr.image_encoder, tr.head):
        for key, (t, members) in Bk.shadow_store(m).items():
            r = 0
            for n, ptr, ver in members:
                p = named[ptr]
                rows = p.shape[0]
                assert torch.equal(t[r:r + rows].reshape(-1), K.cast(p.detach().reshape(-1), torch.bfloat16)), key
                r += rows
                checked += 1
    assert checked > 20
    # an external in-place update invalidates the copy
    w = tr.head.classifier.mlp_text_given_text[0].weight if hasattr(tr.head, "classifier") else None
    p = next(iter(tr.text_encoder.parameters())) if w is None else w
    with torch.no_grad():
        p.mul_(2.0)
    store = Bk.shadow_store(tr.text_encoder if w is None else tr.head)
    stale = [k for k, (t, mem) in store.items() if any(ptr == p.data_ptr() for _, ptr, _ in mem)]
    for k in stale:
        sc = Bk.StepCtx({n: q.detach() for n, q in (tr.text_encoder if w is None else tr.head).named_parameters()},
                        torch.bfloat16, shadows=store)
        names = [n for n, _, _ in store[k][1]]
        assert sc._shadow(k, names) is None


def test_bf16_shadows_registered_again_after_model_replaced():
    """a model built after another was freed (the allocator hands its weight pointers to the new
    model) gets its bf16 weight copies registered — the dead model's SHADOW_OF entries are stale,
    not owners — and AdamW refreshes the new copies (blocks.live_shadow)"""
    import gc
    from mmfd import blocks as Bk

    def registered(tr):
        return sum(len(mem) for m in (tr.text_encoder, tr.image_encoder, tr.head)
                   for key, (t, mem) in Bk.shadow_store(m).items() if not isinstance(key, tuple))

    tr, _ = build_pair("bf16", dropout=0.0)
    tr.step({k: v.cuda() for k, v in tiny_batch(2, seed=50).items()})
    torch.cuda.synchronize()
    n0 = registered(tr)
    assert n0 > 20
    del tr
    gc.collect()
    tr2, _ = build_pair("bf16", dropout=0.0)
    for s in range(2):
        tr2.step({k: v.cuda() for k, v in tiny_batch(2, seed=51 + s).items()})
    torch.cuda.synchronize()
    assert registered(tr2) == n0
    assert all(e[2]() is not None for e in Bk.SHADOW_OF.values())
    from mmfd import kernels as K
    for m in (tr2.text_encoder, tr2.image_encoder, tr2.head):
        P = dict(m.named_parameters())
        for key, (t, members) in Bk.shadow_store(m).items():
            if isinstance(key, tuple):
                continue
            r = 0
            for n, ptr, ver in members:
                rows = P[n].shape[0]
                assert torch.equal(t[r:r + rows].reshape(-1), K.cast(P[n].detach().reshape(-1), torch.bfloat16)), key
                r += rows


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_captured_step_replays_equal_eager_steps(precision):
    """FusionTrainer.capture/replay (the whole step as one HIP graph: dropout seeds advance on the
    device, AdamW's pointer table reserved before the capture and bound after it) matches the same
    number of eager steps, dropout on; new inputs are taken through the static buffers.
    Held to tolerances rather than bits (the eager and captured trainers are separate objects whose
    workspaces and split-K choices need not match), and AdamW turns a rounding-noise gradient (the key
    biases' true gradient is 0) into a +-lr update; parameters are therefore held to 3 steps x lr,
    losses to 1e-5 (fp32) / 1e-3 (bf16)."""
    tr_e, _ = build_pair(precision, dropout=0.1)
    tr_g, _ = build_pair(precision, dropout=0.1)
    b1 = {k: v.cuda() for k, v in tiny_batch(3, seed=41).items()}
    b2 = {k: v.cuda() for k, v in tiny_batch(3, seed=42).items()}
    static = {k: v.clone() for k, v in b1.items()}
    tr_g.capture(static, warmup=2)
    le = [tr_e.step(b1) for _ in range(2)]
    le += [tr_e.step(b1), tr_e.step(b2), tr_e.step(b1)]
    lg = [tr_g.replay().clone(), tr_g.replay(b2).clone(), tr_g.replay(b1).clone()]
    torch.cuda.synchronize()
    tol = 1e-5 if precision == "fp32" else 1e-3
    for a, b in zip(le[2:], lg):
        assert (a.detach() - b).abs().max().item() <= tol * max(1.0, a.abs().max().item())
    lr = tr_e.optimizer.param_groups[0]["lr"]
    for m_e, m_g in ((tr_e.text_encoder, tr_g.text_encoder), (tr_e.image_encoder, tr_g.image_encoder),
                     (tr_e.head, tr_g.head)):
        for (n, p), (_, q) in zip(m_e.named_parameters(), m_g.named_parameters()):
            assert (p - q).abs().max().item() <= 3 * lr + 1e-6, n


@pytest.mark.parametrize("B", [2, 4])
def test_train_step_fp32_split_operand_weight_grads(B):
    """token counts that are whole 64-row tiles (B = 2, 4 pairs of 16 tokens): the weight-gradient
    GEMMs run on split operands and the GELU output / its gradient exist only as epilogue-written
    planes (no fp32 copy) — gradients still match the oracle at the fp32 bounds"""
    tr, ref = build_pair("fp32", dropout=0.0)
    compare_step(tr, ref, tiny_batch(B, seed=21), loss_tol=1e-3, grad_rtol=2e-3)
