"""Training step / loop mirroring the reference's train.py on HIP kernels.

Reference step (train.py:123-188): zero_grad -> (encoders) -> model(X_t, X_i, E_t, E_i) ->
sum_i CrossEntropy(y_i, labels[:, i]) -> backward -> AdamW.step(). Differences, all MI355X-driven:
  * claim and evidence go through each encoder as ONE stacked batch (same weights, same math as the
    reference's two calls at train.py:136-143, twice the GEMM M);
  * the 4 path losses are one kernel; per-step host syncs (.item()/.cpu(), train.py:168-178) are
    removed from the hot loop and only done every `log_every` steps;
  * encoders can be frozen (reference behaviour, train.py:335-340) or fine-tuned (BASELINE config 3);
  * data parallel: one process per GPU, gradients averaged over RCCL (dp.py).
"""
from __future__ import annotations

import argparse
import logging
import os

import torch

from . import kernels as K
from .dataset import synthetic_batch
from .encoders import BertConfig, BertModel, ViTConfig, ViTModel
from .model import MisinformationDetectionModel
from .optim import AdamW

logger = logging.getLogger(__name__)
PATHS = ("text_text", "text_image", "image_text", "image_image")


class _XentFn(torch.autograd.Function):
    """Summed per-path cross entropy (train.py:160-169) -> [total, text_text, text_image,
    image_text, image_image] (fp32, device; 0 for an absent path). Path idx is trained on
    labels[:, idx] whatever the other paths are (train.py:165)."""

    @staticmethod
    def forward(ctx, labels, cols, *logits):
        loss, _ = K.xent_fwd_bwd(list(logits), labels, want_grad=False, cols=cols, n_slots=1 + len(PATHS))
        ctx.cols = cols
        ctx.save_for_backward(labels, *logits)
        return loss

    @staticmethod
    def backward(ctx, g):
        labels, *logits = ctx.saved_tensors
        scale = g[:1].contiguous()  # d total; the per-path entries are for logging only
        _, dl = K.xent_fwd_bwd(logits, labels, want_grad=True, dloss_scale=scale, cols=ctx.cols,
                               n_slots=1 + len(PATHS))
        return (None, None, *dl)


def path_losses(outputs, labels):
    """outputs: ((y_tt, y_ti), (y_it, y_ii)) with None for absent paths (model.py:426-468)."""
    (ytt, yti), (yit, yii) = outputs
    present = [(i, y) for i, y in enumerate((ytt, yti, yit, yii)) if y is not None]
    if not present:
        raise ValueError("path_losses: every path output is None")
    return _XentFn.apply(labels, tuple(i for i, _ in present), *[y for _, y in present])


def category_loss(pred, labels):
    """CrossEntropyLoss(pred, category index) of the single-output heads (factify=True 5-way,
    eval_factify.py:114-139; text_only) -> [total, loss, 0, 0, 0] like path_losses."""
    return _XentFn.apply(labels.reshape(-1), (0,), pred)


class FusionTrainer:
    """Encoders + fusion head + AdamW as one training step."""

    def __init__(self, text_encoder, image_encoder, head, lr=1e-4, freeze_encoders=False, precision="bf16",
                 dp=None):
        self.text_encoder, self.image_encoder, self.head = text_encoder, image_encoder, head
        self.freeze = freeze_encoders
        for m in (text_encoder, image_encoder, head):
            m.set_precision(precision)
        if freeze_encoders:
            for m in (text_encoder, image_encoder):
                m.eval()
                for p in m.parameters():
                    p.requires_grad_(False)
        params = list(head.parameters())
        if not freeze_encoders:
            params = list(text_encoder.parameters()) + list(image_encoder.parameters()) + params
        self.params = params
        self.optimizer = AdamW(params, lr=lr)
        self.dp = dp
        if dp is not None:
            # every replica starts from rank 0's weights (frozen encoders included: all ranks must
            # compute the same function), then the gradient all-reduce overlaps the backward pass
            dp.broadcast_params([p for m in (text_encoder, image_encoder, head) for p in m.parameters()])
            for m in ((head,) if freeze_encoders else (text_encoder, image_encoder, head)):
                m._grad_ready = dp.hook_for(m)

    def step(self, batch):
        self.optimizer.zero_grad(set_to_none=True)
        B = batch["labels"].shape[0]
        with torch.set_grad_enabled(not self.freeze):
            T = self.text_encoder(input_ids=batch["input_ids"], attention_mask=batch["attention_mask"]).last_hidden_state
            I = self.image_encoder(batch["pixel_values"]).last_hidden_state
        outs = self.head(T[:B], I[:B], T[B:], I[B:])
        loss = path_losses(outs, batch["labels"])
        if self.dp is not None:
            self.dp.begin()
        loss[0].backward()
        if self.dp is not None:
            self.dp.finish()
        self.optimizer.step()
        return loss


    @torch.no_grad()
    def predict(self, batch):
        """Dual-encoder + fusion forward in eval mode (BASELINE config 2; the inference of
        evaluate.py:112-164 with batched pairs): ((y_tt, y_ti), (y_it, y_ii)) for claim =
        batch[:B], evidence = batch[B:] of the stacked encoder inputs."""
        mods = (self.text_encoder, self.image_encoder, self.head)
        was = [m.training for m in mods]
        for m in mods:
            m.eval()
        try:
            B = batch["pixel_values"].shape[0] // 2
            T = self.text_encoder(input_ids=batch["input_ids"], attention_mask=batch["attention_mask"]).last_hidden_state
            I = self.image_encoder(batch["pixel_values"]).last_hidden_state
            return self.head(T[:B], I[:B], T[B:], I[B:])
        finally:
            for m, w in zip(mods, was):
                m.train(w)


def build_flagship(device="cuda", precision="bf16", dropout=0.1, freeze_encoders=False, lr=1e-4, dp=None,
                   seed=42, rank=0):
    """bert-base-uncased + ViT-B/16 + the fusion head at 768/768 (BASELINE configs 2-4), random init
    from `seed` (the same on every rank; with `dp` rank 0's weights are broadcast anyway); the
    dropout streams are offset per rank so replicas draw independent masks."""
    torch.manual_seed(seed)
    text = BertModel(BertConfig()).to(device)
    image = ViTModel(ViTConfig()).to(device)
    head = MisinformationDetectionModel(text_input_dim=768, image_input_dim=768, embed_dim=256, num_heads=8,
                                        dropout=dropout, hidden_dim=64, num_classes=3).to(device)
    text.manual_seed(seed + 7919 * rank)
    head.manual_seed(seed + 1 + 7919 * rank)
    return FusionTrainer(text, image, head, lr=lr, freeze_encoders=freeze_encoders, precision=precision, dp=dp)


def parse_args(argv=None):
    """train.py:24-85 flag names, plus --precision / --synthetic / --steps."""
    ap = argparse.ArgumentParser(description="Train misinformation detection model (MI355X)")
    ap.add_argument("--epochs", type=int, default=1)
    ap.add_argument("--batch_size", type=int, default=32)
    ap.add_argument("--lr", type=float, default=1e-4)
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--dropout", type=float, default=0.1)
    ap.add_argument("--freeze_text", action="store_true")
    ap.add_argument("--freeze_image", action="store_true")
    ap.add_argument("--log_every", type=int, default=100)
    ap.add_argument("--output_dir", type=str, default="./results")
    ap.add_argument("--precision", choices=["fp32", "bf16"], default="bf16")
    ap.add_argument("--synthetic", type=int, default=1024, help="number of synthetic Factify-shaped pairs")
    ap.add_argument("--steps", type=int, default=0, help="stop after N steps (0 = full epochs)")
    return ap.parse_args(argv)


def main(args):
    device = torch.device(f"cuda:{args.device}")
    torch.cuda.set_device(device)
    tr = build_flagship(device, args.precision, args.dropout, freeze_encoders=args.freeze_text and args.freeze_image,
                        lr=args.lr, seed=args.seed)
    os.makedirs(args.output_dir, exist_ok=True)
    steps_per_epoch = max(1, args.synthetic // args.batch_size)
    global_step = 0
    for epoch in range(args.epochs):
        for s in range(steps_per_epoch):
            batch = synthetic_batch(args.batch_size, seed=args.seed * 100003 + global_step, device=device)
            loss = tr.step(batch)
            if global_step % args.log_every == 0:
                vals = loss.tolist()
                logger.info("epoch %d step %d total_loss %.4f %s", epoch, global_step, vals[0],
                            " ".join(f"{n}={v:.4f}" for n, v in zip(PATHS, vals[1:])))
            global_step += 1
            if args.steps and global_step >= args.steps:
                break
        torch.save({"global_step": global_step, "epoch": epoch, "model_state_dict": tr.head.state_dict(),
                    "optimizer_state_dict": tr.optimizer.state_dict()},
                   os.path.join(args.output_dir, f"checkpoint-{epoch}-{global_step}.pt"))
        if args.steps and global_step >= args.steps:
            break


if __name__ == "__main__":  # pragma: no cover
    logging.basicConfig(level=logging.INFO)
    main(parse_args())
