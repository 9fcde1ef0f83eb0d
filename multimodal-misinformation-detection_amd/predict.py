"""Single-pair inference: `MisinformationPredictor` of the reference's
evaluate.py:12-196 (and the per-pair voting input of app.py:313-371) on the HIP path.

Two layers:

  * `MisinformationPredictor` — the drop-in for evaluate.py: the reference's constructor
    (`model_path`, device, the model dims, `text_encoder` name; evaluate.py:13-82) and
    `evaluate(claim_text, claim_image_path, evidence_text, evidence_image_path)` (:95-196):
    tokenise both texts to max_length=512 with padding (:112-126), the text encoder on each, the
    images through Resize((256, 256)) + ToTensor + ImageNet Normalize (:71-79, here the HIP
    `ImagePreprocessor("evaluate")`), the image encoder on each, the fusion model, per path softmax
    -> argmax -> label (:82, :169-192). An image that cannot be read makes that modality None
    (:84-92, :141-156): the model then returns None for every path that needs it and evaluate maps
    it to None; any other failure is logged and evaluate returns None, as the reference does.
  * `PairPredictor` — the tensor-level engine under it (token ids, masks, normalised pixels):
    claim and evidence go through each encoder as ONE stacked batch of 2 (same weights), and with
    both images present the whole forward (encoders + fusion head, eval mode) is captured once into a
    HIP graph on static input buffers and replayed per pair (one graph launch instead of ~400 kernel
    launches from Python); a pair with a missing image runs the same kernels eagerly.

The reference loads pretrained DeBERTa-v3-xsmall / Swinv2-base weights by hub name
(evaluate.py:43-48). There is no hub access here: a `text_encoder` / `image_encoder` that is a local
directory holding a `model.safetensors` (or `pytorch_model.bin`) in the HF layout is loaded from it;
the hub names build the architecture with seeded random weights (logged); a ready mmfd encoder
module can be passed instead. The tokenizer is `AutoTokenizer.from_pretrained(text_encoder)` as in
the reference when that resolves offline, else pass `tokenizer=` (an object or a local directory,
as `python -m mmfd.train --tokenizer` does).
"""
from __future__ import annotations

import logging
import os

import torch

from .train import FusionTrainer, load_checkpoint

logger = logging.getLogger(__name__)

IDX_TO_LABEL = {0: "support", 1: "not_enough_information", 2: "refute"}  # evaluate.py:82
PATHS = ("text_text", "text_image", "image_text", "image_image")
DEBERTA_XSMALL = "microsoft/deberta-v3-xsmall"
SWINV2_BASE = "microsoft/swinv2-base-patch4-window8-256"


class PairPredictor:
    """Tensor-level single-pair forward on already-built HIP modules (text encoder, image encoder,
    `mmfd.model.MisinformationDetectionModel`), all on one device."""

    def __init__(self, text_encoder, image_encoder, model, max_length=512, image_size=224, use_graph=True,
                 device=None):
        self.text_encoder, self.image_encoder, self.model = text_encoder, image_encoder, model
        for m in (text_encoder, image_encoder, model):
            m.eval()
        self.device = torch.device(device) if device is not None else next(model.parameters()).device
        if self.device.type != "cuda":
            raise RuntimeError("PairPredictor runs on the HIP device")
        self.max_length, self.image_size = max_length, image_size
        self.use_graph = use_graph
        self.idx_to_label = dict(IDX_TO_LABEL)
        self._graph = None
        L, S = max_length, image_size
        # static inputs of the captured forward: [claim, evidence] stacked
        self._ids = torch.zeros(2, L, dtype=torch.int64, device=self.device)
        self._mask = torch.zeros(2, L, dtype=torch.int64, device=self.device)
        self._px = torch.zeros(2, 3, S, S, dtype=torch.float32, device=self.device)
        self._out = None

    @classmethod
    def from_trainer(cls, trainer: FusionTrainer, **kw):
        return cls(trainer.text_encoder, trainer.image_encoder, trainer.head, **kw)

    @torch.no_grad()
    def _forward(self, have=(True, True)):
        """the fused forward on the static buffers; `have` = (claim image, evidence image) present"""
        T = self.text_encoder(input_ids=self._ids, attention_mask=self._mask).last_hidden_state
        rows = [r for r in range(2) if have[r]]
        Xi = Ei = None
        if rows:
            px = self._px if len(rows) == 2 else self._px[rows[0]:rows[0] + 1]
            I = self.image_encoder(px).last_hidden_state
            Xi = I[:1] if have[0] else None
            Ei = I[len(rows) - 1:] if have[1] else None
        (ytt, yti), (yit, yii) = self.model(T[:1], Xi, T[1:], Ei)
        return ytt, yti, yit, yii

    def _signature(self):
        """(data_ptr, version) of every parameter and buffer the captured forward reads: a graph
        is baked with the addresses of the weight shadows / packed biases built from them, so any
        change (load_state_dict, optimizer outside mmfd's AdamW, .to()) forces a re-capture."""
        return tuple((t.data_ptr(), t._version) for m in (self.text_encoder, self.image_encoder, self.model)
                     for t in (*m.parameters(), *m.buffers()))

    def _capture(self):
        self._sig = self._signature()
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for _ in range(2):  # warm up: one-time casts of the weight shadows, kernel attributes
                self._forward()
        torch.cuda.current_stream(self.device).wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._out = self._forward()
        self._graph = g

    def _load(self, claim_ids, claim_mask, claim_pixels, evidence_ids, evidence_mask, evidence_pixels):
        L = self.max_length
        for row, (ids, mask) in enumerate(((claim_ids, claim_mask), (evidence_ids, evidence_mask))):
            ids = torch.as_tensor(ids).reshape(-1)[:L]  # truncation=True (evaluate.py:113-126)
            mask = torch.ones_like(ids) if mask is None else torch.as_tensor(mask).reshape(-1)[:L]
            self._ids[row].zero_()
            self._mask[row].zero_()
            self._ids[row, :ids.numel()].copy_(ids, non_blocking=True)  # padding="max_length"
            self._mask[row, :mask.numel()].copy_(mask, non_blocking=True)
        for row, px in enumerate((claim_pixels, evidence_pixels)):
            if px is None:
                continue
            px = torch.as_tensor(px)
            if px.dim() == 4:
                px = px[0]
            if tuple(px.shape) != (3, self.image_size, self.image_size):
                raise ValueError(f"pixel tensor must be [3, {self.image_size}, {self.image_size}], got {tuple(px.shape)}")
            self._px[row].copy_(px, non_blocking=True)

    @torch.no_grad()
    def predict_logits(self, claim_ids, claim_mask, claim_pixels, evidence_ids, evidence_mask, evidence_pixels):
        """((y_tt, y_ti), (y_it, y_ii)) logits [1, num_classes] for one pair (model.py:426-468); a
        None pixel tensor = that image is missing: the paths that need it come back None"""
        self._load(claim_ids, claim_mask, claim_pixels, evidence_ids, evidence_mask, evidence_pixels)
        have = (claim_pixels is not None, evidence_pixels is not None)
        if self.use_graph and all(have):
            if self._graph is None or self._sig != self._signature():
                self._graph = None
                self._capture()
            self._graph.replay()
            out = self._out
        else:
            out = self._forward(have)
        ytt, yti, yit, yii = (None if o is None else o.clone() for o in out)
        return (ytt, yti), (yit, yii)

    def process_output(self, output):
        """softmax -> argmax -> {label, confidence, probabilities} (evaluate.py:169-182)."""
        if output is None:
            return None
        probs = torch.softmax(output.float(), dim=-1)[0].cpu()
        idx = int(probs.argmax())
        return {"label": self.idx_to_label[idx], "confidence": float(probs[idx]),
                "probabilities": {self.idx_to_label[i]: float(p) for i, p in enumerate(probs)}}

    def evaluate(self, claim_ids, claim_mask, claim_pixels, evidence_ids, evidence_mask, evidence_pixels,
                 details=False):
        """path -> label (None for a path whose modality is missing) for the four modality paths
        (evaluate.py:184-192); `details` returns the full process_output dicts instead."""
        (ytt, yti), (yit, yii) = self.predict_logits(claim_ids, claim_mask, claim_pixels, evidence_ids,
                                                     evidence_mask, evidence_pixels)
        preds = {p: self.process_output(y) for p, y in zip(PATHS, (ytt, yti, yit, yii))}
        if details:
            return preds
        return {p: (d["label"] if d else None) for p, d in preds.items()}


def _load_local_weights(module, path):
    """HF-layout weights from a local model directory (model.safetensors or pytorch_model.bin; the
    architecture prefix, e.g. "deberta." / "swinv2.", is stripped): True when loaded"""
    if not (path and os.path.isdir(path)):
        return False
    st, pt = os.path.join(path, "model.safetensors"), os.path.join(path, "pytorch_model.bin")
    if os.path.exists(st):
        from safetensors.torch import load_file
        sd = load_file(st)
    elif os.path.exists(pt):
        sd = torch.load(pt, map_location="cpu", weights_only=True)
    else:
        return False
    own = set(module.state_dict())
    fixed = {}
    for k, v in sd.items():
        for pre in ("", "deberta.", "swinv2.", "bert.", "vit.", "model."):
            if k.startswith(pre) and k[len(pre):] in own:
                fixed[k[len(pre):]] = v
                break
    missing = own - set(fixed)
    if missing:
        raise RuntimeError(f"{path}: weights missing for {sorted(missing)[:5]} ...")
    module.load_state_dict(fixed, strict=True)
    return True


def build_text_encoder(name):
    """the reference's AutoModel.from_pretrained(text_encoder) (evaluate.py:43-44) as an mmfd module"""
    from .deberta import DebertaV2Config, DebertaV2Model
    from .encoders import BertConfig, BertModel
    if name == "bert-base-uncased" or (os.path.isdir(str(name)) and "bert" in os.path.basename(str(name)).lower()
                                       and "deberta" not in os.path.basename(str(name)).lower()):
        mod = BertModel(BertConfig())
    else:
        mod = DebertaV2Model(DebertaV2Config())
    if not _load_local_weights(mod, name):
        logger.warning("text encoder %s: pretrained weights are not available offline; seeded random weights of "
                       "the same architecture", name)
    return mod


def build_image_encoder(name=SWINV2_BASE):
    """the reference's Swinv2Model.from_pretrained(swinv2-base-patch4-window8-256) (evaluate.py:45-47)"""
    from .swinv2 import Swinv2Config, Swinv2Model
    mod = Swinv2Model(Swinv2Config())
    if not _load_local_weights(mod, name):
        logger.warning("image encoder %s: pretrained weights are not available offline; seeded random weights of "
                       "the same architecture", name)
    return mod


class MisinformationPredictor:
    """Drop-in for evaluate.py:12 — same constructor arguments and `evaluate` contract. Extra
    keyword-only arguments: `tokenizer` (object or local directory), `text_encoder_module` /
    `image_encoder_module` (ready mmfd encoders), `image_encoder` (name or local directory),
    `precision` ("fp32", the reference's arithmetic, or "bf16"), `use_graph`, `seed` (random
    encoder weights when no local weights exist)."""

    def __init__(self, model_path, device="cuda", embed_dim=256, num_heads=8, dropout=0.1, hidden_dim=64,
                 num_classes=3, mlp_ratio=4.0, text_input_dim=384, image_input_dim=1024, fused_attn=False,
                 text_encoder=DEBERTA_XSMALL, *, tokenizer=None, image_encoder=SWINV2_BASE, text_encoder_module=None,
                 image_encoder_module=None, precision="fp32", use_graph=True, seed=0):
        from .model import MisinformationDetectionModel
        from .preprocess import ImagePreprocessor
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise RuntimeError("MisinformationPredictor runs on the HIP device (device='cuda')")
        logger.info("Loading encoders...")
        self.tokenizer = self._tokenizer(tokenizer, text_encoder)
        torch.manual_seed(seed)
        self.text_encoder = (text_encoder_module or build_text_encoder(text_encoder)).to(self.device)
        self.image_encoder = (image_encoder_module or build_image_encoder(image_encoder)).to(self.device)
        self.model = MisinformationDetectionModel(
            text_input_dim=text_input_dim, image_input_dim=image_input_dim, embed_dim=embed_dim,
            num_heads=num_heads, dropout=dropout, hidden_dim=hidden_dim, num_classes=num_classes,
            mlp_ratio=mlp_ratio, fused_attn=fused_attn).to(self.device)
        logger.info(f"Loading model from {model_path}")
        checkpoint = load_checkpoint(model_path)
        self.model.load_state_dict(checkpoint["model_state_dict"])
        for m in (self.text_encoder, self.image_encoder, self.model):
            m.set_precision(precision)
            m.eval()
        # Resize((256, 256)) + ToTensor + Normalize(ImageNet mean / std) (evaluate.py:71-79)
        self.image_transform = ImagePreprocessor("evaluate", device=self.device)
        self.idx_to_label = dict(IDX_TO_LABEL)
        self._engine = PairPredictor(self.text_encoder, self.image_encoder, self.model, max_length=512,
                                     image_size=self.image_transform.out_hw[0], use_graph=use_graph,
                                     device=self.device)

    @staticmethod
    def _tokenizer(tokenizer, text_encoder):
        from transformers import AutoTokenizer
        if tokenizer is not None and not isinstance(tokenizer, (str, os.PathLike)):
            return tokenizer
        src = tokenizer if tokenizer is not None else text_encoder
        try:
            return AutoTokenizer.from_pretrained(src, local_files_only=True)
        except Exception as e:  # no hub access: the vocabulary must be local
            raise RuntimeError(f"tokenizer for {src!r} is not available offline; pass tokenizer= (a tokenizer object "
                               f"or a local tokenizer directory)") from e

    def process_image(self, image_path):
        """Process image from path to tensor [1, 3, 256, 256] on the device; None when it cannot
        be read (evaluate.py:84-92)."""
        try:
            from PIL import Image
            with Image.open(image_path) as im:
                image = im.convert("RGB")
            return self.image_transform([image])
        except Exception as e:
            logger.error(f"Error processing image {image_path}: {e}")
            return None

    def _tokens(self, text):
        enc = self.tokenizer(text, truncation=True, padding="max_length", max_length=512, return_tensors="pt")
        return enc["input_ids"][0], enc["attention_mask"][0]

    @torch.no_grad()
    def evaluate(self, claim_text, claim_image_path, evidence_text, evidence_image_path):
        """Evaluate a single claim-evidence pair: {path: label or None} (evaluate.py:95-196), or
        None when the evaluation itself fails."""
        try:
            c_ids, c_mask = self._tokens(claim_text)
            e_ids, e_mask = self._tokens(evidence_text)
            claim_image = self.process_image(claim_image_path)
            evidence_image = self.process_image(evidence_image_path)
            if claim_image is None:
                logger.warning("Claim image processing failed, setting embedding to None")
            if evidence_image is None:
                logger.warning("Evidence image processing failed, setting embedding to None")
            return self._engine.evaluate(c_ids, c_mask, claim_image, e_ids, e_mask, evidence_image)
        except Exception as e:
            logger.error(f"Error during evaluation: {e}")
            return None

    def predict_logits(self, claim_text, claim_image_path, evidence_text, evidence_image_path):
        """the four paths' logits ((y_tt, y_ti), (y_it, y_ii)) of `evaluate`'s forward (None for a
        path whose image is missing)"""
        c_ids, c_mask = self._tokens(claim_text)
        e_ids, e_mask = self._tokens(evidence_text)
        return self._engine.predict_logits(c_ids, c_mask, self.process_image(claim_image_path), e_ids, e_mask,
                                           self.process_image(evidence_image_path))
