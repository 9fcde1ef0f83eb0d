"""The chunked oracle step with dropout on: oracle.train_step.chunked_loss_grads
binds each chunk's dropout masks to the chunk's WHOLE-BATCH rows (oracle.dropout_hash.Drop), so the
loss and gradients of a batch computed in chunks equal those of the same batch in one piece — the
masks the HIP kernels draw for the whole batch at once. CPU only (tiny shapes)."""
import numpy as np
import torch

from oracle.dropout_hash import Drop, keep_mask, keep_mask_rows, salt_of
from oracle.train_step import chunked_loss_grads
from tests.smoke_impl import TINY, build_modules, oracle_cfgs, tiny_batch


def test_keep_mask_rows_is_the_whole_batch_mask():
    shape = (6, 3, 5, 7)
    full = keep_mask(11, salt_of("x"), shape, 0.1)
    rows = np.array([4, 1, 5])
    part = keep_mask_rows(11, salt_of("x"), (3,) + shape[1:], 0.1, rows)
    assert (part == full[rows]).all()
    # token-major views of batch-major tensors ([B*L, D]) map the same way
    part2 = keep_mask_rows(11, salt_of("x"), (3 * 3 * 5, 7), 0.1, rows)
    assert (part2.reshape(3, 3, 5, 7) == full[rows]).all()


class _ChunkLocal(Drop):
    """round 4's behaviour: every chunk hashed its own flat indices (with_rows ignored)"""

    def with_rows(self, rows):
        return self


def test_chunked_dropout_step_equals_whole_batch_step():
    _, _, _, states = build_modules(dropout=0.1, cfg=TINY, seed=5)
    batch = tiny_batch(4, cfg=TINY, seed=3)
    bcfg, vcfg = oracle_cfgs(TINY)
    kw = dict(bert_cfg=bcfg, vit_cfg=vcfg, num_heads=TINY["head_heads"])
    whole = chunked_loss_grads(*states, batch, chunk=4, drop=Drop(7, 0.1), drop_head=Drop(8, 0.1), **kw)
    # gradients that are zero in exact arithmetic (attention key biases: softmax is shift invariant)
    # are fp32 noise either way: every tensor is judged against at least 1e-3 of the largest gradient
    floor = 1e-3 * max(g.abs().max().item() for g in whole[2].values() if g is not None)
    for chunk in (1, 3):
        part = chunked_loss_grads(*states, batch, chunk=chunk, drop=Drop(7, 0.1), drop_head=Drop(8, 0.1), **kw)
        assert abs(part[0].item() - whole[0].item()) <= 1e-6, (chunk, part[0].item(), whole[0].item())
        for k, g in whole[2].items():
            if g is None:
                assert part[2][k] is None, k
                continue
            err = (part[2][k] - g).abs().max().item() / max(g.abs().max().item(), floor)
            assert err <= 1e-4, (chunk, k, err)
    # the mapping matters: chunk-local masks give another loss
    local = chunked_loss_grads(*states, batch, chunk=1, drop=_ChunkLocal(7, 0.1), drop_head=_ChunkLocal(8, 0.1), **kw)
    assert abs(local[0].item() - whole[0].item()) > 1e-4


def test_attn_keep_mask_pairs_rows_and_rate():
    """attention masks (one hash per key pair, 16-bit halves): whole-batch rows map like keep_mask_rows,
    odd Lk pads the last pair, the keep rate is 1 - p within sampling error, and the two halves of a
    pair are not correlated"""
    from oracle.dropout_hash import attn_keep_mask, drop_threshold16
    assert drop_threshold16(0.1) == 6554 and drop_threshold16(0.0) == 0 and drop_threshold16(1.0) == 65536
    full = attn_keep_mask(5, salt_of("a.attn"), (5, 3, 7, 13), 0.1)
    rows = np.array([3, 0, 4])
    assert (attn_keep_mask(5, salt_of("a.attn"), (3, 3, 7, 13), 0.1, rows) == full[rows]).all()
    big = attn_keep_mask(11, salt_of("b.attn"), (4, 8, 64, 128), 0.1)
    rate = big.mean()
    assert abs(rate - 0.9) < 0.004, rate
    even, odd = big[..., 0::2].astype(np.float64), big[..., 1::2].astype(np.float64)
    corr = ((even - even.mean()) * (odd - odd.mean())).mean() / (even.std() * odd.std())
    assert abs(corr) < 0.01, corr
    assert not attn_keep_mask(1, 2, (1, 1, 4, 6), 1.0).any() and attn_keep_mask(1, 2, (1, 1, 4, 6), 0.0).all()


def test_bench_trajectory_fixture_starts_at_the_one_step_fixture():
    """tests/golden/config3_bs256_p01_traj.npz (30 oracle AdamW steps of the bench recipe, the
    reference for bench.py's final_loss) begins with the one-step fixture's loss vector and records
    the recipe it was made from"""
    import os
    g = os.path.join(os.path.dirname(__file__), "golden")
    one = np.load(os.path.join(g, "config3_bs256_p01.npz"))
    traj = np.load(os.path.join(g, "config3_bs256_p01_traj.npz"))
    assert str(traj["recipe"]) == "bench" == str(one["recipe"])
    steps = traj["loss_steps"]
    assert steps.shape == (30, 5) and np.isfinite(steps).all()
    assert np.abs(steps[0] - one["loss"]).max() <= 1e-12
    assert steps[-1, 0] < steps[0, 0]  # the fixed batch is being fitted
