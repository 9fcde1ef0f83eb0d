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

import numpy as np
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


def _numpy_scalar_globals():
    """the pickle globals a numpy scalar needs (np.float64 / np.int64 as np.mean and sklearn leave
    them): the scalar reconstructor under its numpy-2 and numpy-1 module paths and the dtype classes"""
    import numpy as np
    scalar = np._core.multiarray.scalar
    allow = [scalar, (scalar, "numpy.core.multiarray.scalar"), np.dtype]
    for t in (np.float64, np.float32, np.float16, np.int64, np.int32, np.bool_):
        allow.append(type(np.dtype(t)))
    return allow


def load_checkpoint(path, map_location="cpu"):
    """torch.load(weights_only=True) of a reference checkpoint. The reference's best_model.pt
    (train.py:413-428) stores the best metric as a numpy scalar (np.mean of the F1s), which the
    weights-only unpickler refuses by default: only numpy's scalar reconstructor and dtype classes
    are allowed in addition — still no code from the file runs."""
    with torch.serialization.safe_globals(_numpy_scalar_globals()):
        return torch.load(path, map_location=map_location, weights_only=True)


class FusionTrainer:
    """Encoders + fusion head + AdamW as one training step (train.py:123-188).

    Batches come in two forms (mmfd.dataset.stack_pairs): encoder inputs (input_ids /
    attention_mask [2B, L] and pixel_values [2B, 3, S, S], claims first) or pre-computed encoder
    outputs (claim_text_embeds / doc_text_embeds / claim_image_embeds / doc_image_embeds, the
    reference's --pre_embed mode, train.py:127-132; the encoders may then be None). Each encoder
    is frozen (eval, no grad: the reference's behaviour, train.py:335-340) or fine-tuned
    (BASELINE config 3) on its own: freeze_text / freeze_image (default: freeze_encoders)."""

    def __init__(self, text_encoder, image_encoder, head, lr=1e-4, freeze_encoders=False, precision="bf16",
                 dp=None, freeze_text=None, freeze_image=None):
        self.text_encoder, self.image_encoder, self.head = text_encoder, image_encoder, head
        self.freeze_text = freeze_encoders if freeze_text is None else bool(freeze_text)
        self.freeze_image = freeze_encoders if freeze_image is None else bool(freeze_image)
        self.freeze = self.freeze_text and self.freeze_image
        for m in (text_encoder, image_encoder, head):
            if m is not None:
                m.set_precision(precision)
        trained = [head]
        for m, frozen in ((text_encoder, self.freeze_text), (image_encoder, self.freeze_image)):
            if m is None:
                continue
            if frozen:
                m.eval()
                for p in m.parameters():
                    p.requires_grad_(False)
            else:
                trained.insert(len(trained) - 1, m)
        self.params = [p for m in trained for p in m.parameters()]
        self.optimizer = AdamW(self.params, lr=lr)
        self.dp = dp
        # text / image encoders on two streams (see _encode)
        self.concurrent = os.environ.get("MMFD_SERIAL_ENCODERS") != "1"
        if dp is not None:
            # every replica starts from rank 0's weights (frozen encoders included: all ranks must
            # compute the same function), then the gradient all-reduce overlaps the backward pass
            dp.broadcast_params([p for m in (text_encoder, image_encoder, head) if m is not None
                                 for p in m.parameters()])
            for m in trained:
                m._grad_ready = dp.hook_for(m)

    def _device(self):
        return next(self.head.parameters()).device

    def _side_stream(self, dev):
        st = getattr(self, "_side", None)
        if st is None or st.device != dev:
            st = self._side = torch.cuda.Stream(device=dev)
        return st

    def _encode(self, batch, dev):
        """(T, I): the text and image encoders on the stacked claim/evidence inputs (frozen ones
        without autograd). In a single process the two encoders run on two HIP streams — they are
        independent until the head, so one's MFMA main loops overlap the other's HBM-bound
        epilogues, attention and LayerNorms and fill its last-round GEMM tiles; autograd runs each
        encoder's backward on its forward stream and joins them before the optimizer (the DP
        all-reduce buckets gradients per stream, mmfd.dp)."""
        ids = batch["input_ids"].to(dev, non_blocking=True)
        mask = batch["attention_mask"].to(dev, non_blocking=True)
        pix = batch["pixel_values"].to(dev, non_blocking=True)
        conc = self.concurrent
        main = torch.cuda.current_stream(dev)
        if conc:
            side = self._side_stream(dev)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                with torch.set_grad_enabled(torch.is_grad_enabled() and not self.freeze_text):
                    T = self.text_encoder(input_ids=ids, attention_mask=mask).last_hidden_state
        else:
            with torch.set_grad_enabled(torch.is_grad_enabled() and not self.freeze_text):
                T = self.text_encoder(input_ids=ids, attention_mask=mask).last_hidden_state
        with torch.set_grad_enabled(torch.is_grad_enabled() and not self.freeze_image):
            I = self.image_encoder(pix).last_hidden_state
        if conc:
            main.wait_stream(side)
            T.record_stream(main)
        return T, I

    def features(self, batch):
        """(X_t, X_i, E_t, E_i) for the head: the batch's pre-computed embeddings, or the encoders
        on the stacked claim/evidence inputs (frozen ones without autograd)"""
        dev = self._device()
        if "claim_text_embeds" in batch:
            return tuple(batch[k].to(dev, non_blocking=True) for k in
                         ("claim_text_embeds", "claim_image_embeds", "doc_text_embeds", "doc_image_embeds"))
        B = batch["labels"].shape[0]
        T, I = self._encode(batch, dev)
        return T[:B], I[:B], T[B:], I[B:]

    def loss(self, outs, labels):
        if self.head.factify or self.head.text_only:
            return category_loss(outs[0], labels)
        return path_losses(outs, labels)

    def _head_forward(self, batch):
        """the head on the batch's features; encoder outputs go in stacked (forward_pairs), so their
        gradients come back as one tensor per encoder"""
        if "claim_text_embeds" in batch or self.text_encoder is None or self.image_encoder is None:
            return self.head(*self.features(batch))
        T, I = self._encode(batch, self._device())
        return self.head.forward_pairs(T, I, batch["labels"].shape[0])

    def step(self, batch, return_outputs=False):
        """one optimizer step; returns the device loss vector [total, tt, ti, it, ii] (and the
        logits with return_outputs)"""
        self.optimizer.zero_grad(set_to_none=True)
        outs = self._head_forward(batch)
        loss = self.loss(outs, batch["labels"].to(self._device(), non_blocking=True))
        if self.dp is not None:
            self.dp.begin()
        # d total / d loss = [1, 0, 0, 0, 0]: one resident vector, no per-step fill kernels
        g = getattr(self, "_dtotal", None)
        if g is None or g.device != loss.device:
            g = self._dtotal = torch.tensor([1.0] + [0.0] * (loss.numel() - 1), device=loss.device)
        torch.autograd.backward(loss, g)
        if self.dp is not None:
            self.dp.finish()
        self.optimizer.step()
        # detached results: a returned loss / logits still holding their grad_fn would keep this
        # step's autograd graph — and the AccumulateGrad nodes of every parameter, bound to the
        # streams of this step — alive into the next step, where the text encoder's backward runs
        # on the other stream (torch's "AccumulateGrad node's stream does not match" warning and
        # an extra cross-stream synchronisation)
        loss = loss.detach()
        if return_outputs:
            return loss, _detach_outs(outs)
        return loss

    # ---- the whole step as one HIP graph ------------------------------------------------------------
    def capture(self, batch, warmup=2):
        """Capture one full training step (encoders + head forward, backward, AdamW) on `batch` into
        a HIP graph: replay() then runs it with one launch and no per-kernel host work (the dropout
        seeds advance on the device, AdamW's pointer table is bound after capture). `batch` tensors
        are the graph's static inputs: refill them in place (or pass a batch to replay) between
        replays. With data parallelism (`dp`) the gradient all-reduce is captured too: the per-
        stream bucket packs, the RCCL all_reduce kernels (ProcessGroupNCCL keeps captured work out of
        its watchdog) and finish()'s wait + unpack become nodes of the same graph; the buckets were
        allocated by the eager warm-up steps, so the graph reads and writes fixed addresses.

        No timing assumption (round 4 slept 0.5 s here): the captured all-reduces go to the DP
        object's dedicated capture group, whose RCCL stream never carried an eager collective, and
        the capture runs in the thread-local error mode, under which the watchdog thread's event
        queries of the eager collectives (default group, never captured) stay legal (mmfd.dp).
        `first_loss` keeps the loss vector of the first warm-up step (the first optimizer step of
        this trainer when it is fresh)."""
        self._static = batch
        if self.dp is not None and self.dp._active():
            self.dp.capture_group()  # collective: created before the warm-up steps (mmfd.dp)
        s = torch.cuda.Stream(device=self._device())
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for i in range(warmup):  # optimizer state, weight shadows, kernel attributes
                loss = self.step(batch)
                if i == 0:
                    self.first_loss = loss.clone()
        torch.cuda.current_stream().wait_stream(s)
        dp_on = self.dp is not None and self.dp._active()
        if dp_on:
            torch.cuda.synchronize()
            self.dp.use_capture_group(True)
        self.optimizer.prepare_capture()  # pointer tables outside the graph's memory pool
        g = torch.cuda.CUDAGraph()
        try:
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                self._graph_loss = self.step(batch)
        finally:
            if dp_on:
                self.dp.use_capture_group(False)
        self.optimizer.finalize_capture()
        self._graph = g
        return self

    def verify_capture(self, batch=None):
        """Self-check of the captured data-parallel step: one replay, then every rank compares a
        checksum of all its gradients and parameters with the others (mmfd.dp.GradAllReduce.
        consistent: MIN == MAX over the ranks). The ranks train on different batches, so the
        averaged gradients — and the parameters AdamW moves with them — are bitwise equal on every
        rank only if the captured all-reduce really ran. True without data parallelism."""
        if self.dp is None or not self.dp._active():
            return True
        self.replay(batch)
        torch.cuda.synchronize()
        return self.dp.consistent(self.dp_state())

    def dp_state(self):
        """the tensors every rank must agree on after a data-parallel step: the trained parameters'
        gradients, then all parameters"""
        return [p.grad for p in self.params] + [p for p in self.params]

    def resync_state(self, src=0):
        """Every rank takes rank `src`'s parameters and AdamW state (moments and step counters): the
        recovery after a captured DP step that failed verify_capture — its verifying replay already
        ran AdamW on gradients that were not averaged across the ranks, so the replicas (and their
        moments) diverged, and eager DP steps average gradients but never re-sync parameters. The
        in-place parameter copies bump the version counters, so the bf16 weight shadows are re-cast."""
        if self.dp is None or not self.dp._active():
            return
        torch.cuda.synchronize()
        state = []
        for p in self.params:
            st = self.optimizer.state.get(p) if self.optimizer is not None else None
            if st:
                state += [st.get("exp_avg"), st.get("exp_avg_sq"), st.get("step")]
        self.dp.broadcast_tensors(list(self.params) + state, src=src)
        torch.cuda.synchronize()

    def release_graph(self):
        """drop the captured step and its private memory pool (eager steps afterwards)"""
        self._graph = self._graph_loss = None
        torch.cuda.synchronize()
        torch.cuda.empty_cache()

    def replay(self, batch=None):
        """one captured training step; returns the (static) device loss vector"""
        if batch is not None and batch is not self._static:
            for k, v in self._static.items():
                if torch.is_tensor(v):
                    v.copy_(batch[k], non_blocking=True)
        self._graph.replay()
        return self._graph_loss

    @torch.no_grad()
    def predict(self, batch):
        """Dual-encoder + fusion forward in eval mode (BASELINE config 2; the inference of
        evaluate.py:112-164 with batched pairs): ((y_tt, y_ti), (y_it, y_ii)) for claim =
        batch[:B], evidence = batch[B:] of the stacked encoder inputs (or the batch's embeddings)."""
        mods = [m for m in (self.text_encoder, self.image_encoder, self.head) if m is not None]
        was = [m.training for m in mods]
        for m in mods:
            m.eval()
        try:
            if "labels" not in batch and "claim_text_embeds" not in batch:
                batch = dict(batch, labels=torch.empty(batch["pixel_values"].shape[0] // 2))
            return self._head_forward(batch)
        finally:
            for m, w in zip(mods, was):
                m.train(w)


def capture_dp_step(tr, batch, warmup, device, log=logger.info):
    """Capture the data-parallel step on every rank and agree on it (bench.py with MMFD_DP_GRAPH=1).
    Returns (graphed, check): every rank gets the same answer. A rank whose capture raises goes
    eager, and then all do (MIN over the ranks of a success flag); a captured step whose replay
    leaves the ranks with different gradients or parameters (FusionTrainer.verify_capture: the
    captured all-reduce did not run, or not in step) is released on every rank as well."""
    import torch.distributed as dist
    ok = True
    try:
        tr.capture(batch, warmup=warmup)
    except Exception as e:  # a stack that refuses to capture the collectives
        log(f"DP step capture failed ({e!r}); eager steps")
        ok = False
    flag = torch.tensor([1 if ok else 0], device=device, dtype=torch.int32)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    if int(flag.item()) == 0:
        tr.release_graph()
        return False, "capture failed on a rank: eager steps"
    if not tr.verify_capture():
        log("captured DP step failed the cross-rank checksum; rank 0's parameters and AdamW state "
            "re-broadcast, eager steps on every rank")
        tr.release_graph()
        tr.resync_state(src=0)  # the verifying replay stepped AdamW on un-averaged gradients
        return False, "captured all-reduce MISMATCH: state re-synced from rank 0, eager steps"
    return True, "captured all-reduce verified"


def _detach_outs(o):
    if torch.is_tensor(o):
        return o.detach()
    if isinstance(o, (tuple, list)):
        return type(o)(_detach_outs(x) for x in o)
    return o


def flagship_modules(seed=42, dropout=0.1, encoder_dropout=None):
    """(text, image, head) of the flagship on the CPU, initialised from `seed` exactly as
    build_flagship does (the weights tests/golden/make_config3_bs256.py gives the oracle)"""
    torch.manual_seed(seed)
    bc = BertConfig() if encoder_dropout is None else BertConfig(hidden_dropout_prob=encoder_dropout,
                                                                  attention_probs_dropout_prob=encoder_dropout)
    text = BertModel(bc)
    image = ViTModel(ViTConfig())
    head = MisinformationDetectionModel(text_input_dim=768, image_input_dim=768, embed_dim=256, num_heads=8,
                                        dropout=dropout, hidden_dim=64, num_classes=3)
    return text, image, head


def flagship_dropout_seeds(seed=42, rank=0):
    """(text encoder, head) dropout seeds of build_flagship's rank `rank` (advanced by one per step)"""
    return seed + 7919 * rank, seed + 1 + 7919 * rank


def build_flagship(device="cuda", precision="bf16", dropout=0.1, freeze_encoders=False, lr=1e-4, dp=None,
                   seed=42, rank=0, encoder_dropout=None):
    """bert-base-uncased + ViT-B/16 + the fusion head at 768/768 (BASELINE configs 2-4), random init
    from `seed` (the same on every rank; with `dp` rank 0's weights are broadcast anyway); the
    dropout streams are offset per rank so replicas draw independent masks. `dropout` is the head's
    (model.py dropout=0.1); the encoders keep their HF configs' own (BERT 0.1, ViT 0.0).
    `encoder_dropout` overrides BERT's only: ViT-B/16 trains without dropout, and mmfd's ViT
    implements only that configuration (a ViTConfig with dropout raises in training)."""
    text, image, head = (m.to(device) for m in flagship_modules(seed, dropout, encoder_dropout))
    st, sh = flagship_dropout_seeds(seed, rank)
    text.manual_seed(st)
    head.manual_seed(sh)
    return FusionTrainer(text, image, head, lr=lr, freeze_encoders=freeze_encoders, precision=precision, dp=dp)


def parse_args(argv=None):
    """train.py:24-85 (same flags and defaults), plus mmfd's: --precision, --image_encoder,
    --synthetic, --steps, --init_checkpoint, --tokenizer, --world_size-free DP via torchrun."""
    ap = argparse.ArgumentParser(description="Train misinformation detection model (MI355X)")
    ap.add_argument("--epochs", type=int, default=50)
    ap.add_argument("--batch_size", type=int, default=32)
    ap.add_argument("--lr", type=float, default=1e-4)
    ap.add_argument("--num_workers", type=int, default=8)
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--embed_dim", type=int, default=256)
    ap.add_argument("--num_heads", type=int, default=8)
    ap.add_argument("--dropout", type=float, default=0.1)
    ap.add_argument("--hidden_dim", type=int, default=64)
    ap.add_argument("--num_classes", type=int, default=3)
    ap.add_argument("--mlp_ratio", type=float, default=4.0)
    ap.add_argument("--fused_attn", action="store_true", help="accepted: eager and SDPA are one kernel here")
    ap.add_argument("--train_data", type=str, default="./data/preprocessed/train.csv")
    ap.add_argument("--val_data", type=str)
    ap.add_argument("--text_encoder", type=str, default="microsoft/deberta-v3-xsmall",
                    help="microsoft/deberta-v3-xsmall (frozen) or bert-base-uncased")
    ap.add_argument("--output_dir", type=str, default="./results")
    ap.add_argument("--save_every", type=int, default=2000)
    ap.add_argument("--log_every", type=int, default=100)
    ap.add_argument("--wandb_project", type=str, default="misinformation-detection", help="accepted; metrics go to "
                    "<output_dir>/metrics.jsonl under the reference's wandb keys")
    ap.add_argument("--wandb_entity", type=str, default=None)
    ap.add_argument("--freeze_text", action="store_true")
    ap.add_argument("--freeze_image", action="store_true")
    ap.add_argument("--validate_every_epoch", action="store_true")
    ap.add_argument("--save_best", action="store_true")
    ap.add_argument("--best_metric", type=str, default="avg_f1",
                    choices=["avg_f1", "avg_accuracy", "text_text_f1", "text_image_f1", "image_text_f1",
                             "image_image_f1"])
    ap.add_argument("--log_confusion_matrix", action="store_true")
    ap.add_argument("--log_confusion_matrix_every", type=int, default=1000)
    ap.add_argument("--pre_embed", action="store_true")
    ap.add_argument("--text_input_dim", type=int, default=384)
    ap.add_argument("--image_input_dim", type=int, default=1024)
    # mmfd
    ap.add_argument("--image_encoder", type=str, default="microsoft/swinv2-base-patch4-window8-256",
                    help="microsoft/swinv2-base-patch4-window8-256 (frozen) or google/vit-base-patch16-224")
    ap.add_argument("--precision", choices=["fp32", "bf16"], default="fp32")
    ap.add_argument("--synthetic", type=int, default=0,
                    help="train on N synthetic Factify-shaped pairs instead of --train_data")
    ap.add_argument("--steps", type=int, default=0, help="stop after N optimizer steps (0 = all epochs)")
    ap.add_argument("--init_checkpoint", type=str, default=None, help="model_state_dict to start from")
    ap.add_argument("--tokenizer", type=str, default=None, help="local HF tokenizer directory for raw text")
    return ap.parse_args(argv)


TEXT_ENCODERS = ("microsoft/deberta-v3-xsmall", "bert-base-uncased")
IMAGE_ENCODERS = ("microsoft/swinv2-base-patch4-window8-256", "google/vit-base-patch16-224")


def build_encoders(args, device):
    """the encoders of train.py:329-340 (random init: no hub download here). DeBERTa-v3 / Swinv2
    are inference encoders in mmfd and therefore always frozen, as in the reference; bert-base /
    ViT-B/16 train unless --freeze_text / --freeze_image."""
    if args.text_encoder == "microsoft/deberta-v3-xsmall":
        from .deberta import DebertaV2Config, DebertaV2Model
        text, text_frozen = DebertaV2Model(DebertaV2Config()), True
    elif args.text_encoder == "bert-base-uncased":
        text, text_frozen = BertModel(BertConfig()), args.freeze_text
    else:
        raise ValueError(f"--text_encoder must be one of {TEXT_ENCODERS}")
    if args.image_encoder == "microsoft/swinv2-base-patch4-window8-256":
        from .swinv2 import Swinv2Config, Swinv2Model
        image, image_frozen = Swinv2Model(Swinv2Config()), True
    elif args.image_encoder == "google/vit-base-patch16-224":
        image, image_frozen = ViTModel(ViTConfig()), args.freeze_image
    else:
        raise ValueError(f"--image_encoder must be one of {IMAGE_ENCODERS}")
    return text.to(device), image.to(device), text_frozen, image_frozen


def _metrics(preds, labels, prefix):
    """train.py:191-214 / 296-303: accuracy, weighted F1 and per-class F1 per path (sklearn)"""
    from sklearn.metrics import accuracy_score, f1_score
    out = {}
    for path in preds:
        if not preds[path]:
            continue
        y, p = labels[path], preds[path]
        out[f"{prefix}{path}_accuracy"] = float(accuracy_score(y, p))
        out[f"{prefix}{path}_f1"] = float(f1_score(y, p, average="weighted"))
        for i, f in enumerate(f1_score(y, p, average=None)):
            out[f"{prefix}{path}_class{i}_f1"] = float(f)
    return out


def _collect(outs, labels, preds, labs, factify):
    """host-side argmax of a step's logits (only at log time: no per-step device sync)"""
    labels = labels.cpu()
    if factify:
        preds.setdefault("category", []).extend(outs[0].argmax(-1).cpu().tolist())
        labs.setdefault("category", []).extend(labels.reshape(-1).tolist())
        return
    for idx, (path, y) in enumerate(zip(PATHS, (y for pr in outs for y in pr))):
        if y is not None:
            preds.setdefault(path, []).extend(y.argmax(-1).cpu().tolist())
            labs.setdefault(path, []).extend(labels[:, idx].tolist())


@torch.no_grad()
def evaluate(trainer, loader):
    """validation pass (the intent of train.py:248-309, whose model.tokenizer / raw-image inputs
    cannot run): per-path mean loss + accuracy / F1"""
    n, tot = 0, None
    preds, labs = {}, {}
    for batch in loader:
        outs = trainer.predict(batch)
        labels = batch["labels"].to(trainer._device())
        loss = trainer.loss(outs, labels)
        tot = loss if tot is None else tot + loss
        n += 1
        _collect(outs, labels, preds, labs, trainer.head.factify or trainer.head.text_only)
    vals = (tot / max(n, 1)).tolist() if tot is not None else [0.0] * 5
    return {p: v for p, v in zip(PATHS, vals[1:])}, _metrics(preds, labs, "")


def _save(path, **state):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    torch.save(state, path)


def main(args):
    """train.py:311-434 on the HIP path"""
    import functools
    import json
    import torch.distributed as dist
    from torch.utils.data import DataLoader
    from .dataset import MisinformationDataset, SyntheticFactifyDataset, get_dataloader, stack_pairs

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(args.device)))
    device = torch.device(f"cuda:{local}")
    torch.cuda.set_device(device)
    dp = None
    if world > 1:
        from .dp import GradAllReduce
        dist.init_process_group("nccl", device_id=device)
        dp = GradAllReduce()
    os.makedirs(args.output_dir, exist_ok=True)
    torch.manual_seed(args.seed)  # set_seed (train.py:97-101)
    text = image = None
    ft = fi = True
    if not args.pre_embed:
        text, image, ft, fi = build_encoders(args, device)
    head = MisinformationDetectionModel(text_input_dim=args.text_input_dim, image_input_dim=args.image_input_dim,
                                        embed_dim=args.embed_dim, num_heads=args.num_heads, dropout=args.dropout,
                                        hidden_dim=args.hidden_dim, num_classes=args.num_classes,
                                        mlp_ratio=args.mlp_ratio, fused_attn=args.fused_attn)
    if args.init_checkpoint:
        ck = load_checkpoint(args.init_checkpoint)
        head.load_state_dict(ck.get("model_state_dict", ck))
    head = head.to(device)
    head.manual_seed(args.seed + 7919 * rank)
    if text is not None and hasattr(text, "manual_seed"):
        text.manual_seed(args.seed + 1 + 7919 * rank)
    tr = FusionTrainer(text, image, head, lr=args.lr, precision=args.precision, dp=dp, freeze_text=ft,
                       freeze_image=fi)
    tok = None
    if args.tokenizer:
        from transformers import AutoTokenizer
        tok = AutoTokenizer.from_pretrained(args.tokenizer)
    collate = functools.partial(stack_pairs, tokenizer=tok)
    if args.synthetic:
        size = 256 if "swinv2" in args.image_encoder else 224
        ds = SyntheticFactifyDataset(args.synthetic, seq_len=128, image_size=size, seed=args.seed, ragged=True)
        workers = 0
    else:
        ds = MisinformationDataset(args.train_data, pre_embed=args.pre_embed)
        workers = args.num_workers
    # data parallel: each rank draws its own shard of every epoch (DistributedSampler)
    sampler = torch.utils.data.distributed.DistributedSampler(ds, world, rank, shuffle=True, seed=args.seed) \
        if world > 1 else None
    loader = DataLoader(ds, batch_size=args.batch_size, shuffle=sampler is None, sampler=sampler,
                        num_workers=workers, pin_memory=True, collate_fn=collate)
    val_loader = None
    if args.validate_every_epoch:
        if not args.val_data:
            raise ValueError("--val_data must be specified when --validate_every_epoch is set")
        val_loader = get_dataloader(args.val_data, batch_size=args.batch_size, shuffle=False,
                                    num_workers=args.num_workers, pre_embed=args.pre_embed, collate_fn=collate)
    log = open(os.path.join(args.output_dir, "metrics.jsonl"), "a") if rank == 0 else None
    global_step, best = 0, float("-inf")
    single = tr.head.factify or tr.head.text_only  # train.py always builds the 4-path head
    for epoch in range(args.epochs):
        if sampler is not None:
            sampler.set_epoch(epoch)
        preds, labs, pending = {}, {}, []
        for batch in loader:
            loss, outs = tr.step(batch, return_outputs=True)
            pending.append((loss.detach(), outs, batch["labels"]))
            if global_step % args.log_every == 0:
                for _, o_, y_ in pending:
                    _collect(o_, y_, preds, labs, single)
                vals = loss.tolist()
                rec = {"train/total_loss": vals[0], **{f"train/{p}_loss": v for p, v in zip(PATHS, vals[1:])},
                       "train/learning_rate": args.lr, "train/step": global_step, "epoch": epoch,
                       **_metrics(preds, labs, "train/")}
                logger.info("epoch %d step %d total_loss %.4f", epoch, global_step, vals[0])
                if log:
                    log.write(json.dumps(rec) + "\n")
                    log.flush()
                preds, labs = {}, {}
                pending = []
            elif len(pending) > args.log_every:
                pending = pending[-args.log_every:]
            if global_step % args.save_every == 0 and rank == 0:  # train.py:234-242
                _save(os.path.join(args.output_dir, f"checkpoint-{epoch}-{global_step}", "model.pt"),
                      global_step=global_step, epoch=epoch, model_state_dict=tr.head.state_dict(),
                      optimizer_state_dict=tr.optimizer.state_dict())
            global_step += 1
            if args.steps and global_step >= args.steps:
                break
        if val_loader is not None:
            vl, vm = evaluate(tr, val_loader)
            if log:
                log.write(json.dumps({"val/loss": sum(vl.values()) / len(vl), **{f"val/{k}_loss": v for k, v in vl.items()},
                                      **{f"val/{k}": v for k, v in vm.items()}, "epoch": epoch,
                                      "global_step": global_step}) + "\n")
            if args.save_best and rank == 0:  # train.py:409-428
                if args.best_metric == "avg_f1":
                    cur = float(np.mean([v for k, v in vm.items() if k.endswith("_f1") and "class" not in k]))
                elif args.best_metric == "avg_accuracy":
                    cur = float(np.mean([v for k, v in vm.items() if "accuracy" in k]))
                else:
                    cur = vm.get(args.best_metric)
                if cur is not None and cur > best:
                    best = cur
                    _save(os.path.join(args.output_dir, "best_model.pt"), epoch=epoch, global_step=global_step,
                          model_state_dict=tr.head.state_dict(), optimizer_state_dict=tr.optimizer.state_dict(),
                          **{args.best_metric: best})
        if args.steps and global_step >= args.steps:
            break
    if log:
        log.close()
    if world > 1:
        dist.destroy_process_group()
    return tr, global_step


if __name__ == "__main__":  # pragma: no cover
    logging.basicConfig(level=logging.INFO)
    main(parse_args())
