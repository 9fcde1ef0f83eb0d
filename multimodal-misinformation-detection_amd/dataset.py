"""Mirror of src/model/dataset.py: label maps, Dataset / DataLoader factory (same dict keys), plus a
synthetic Factify-shaped pair generator for benchmarks and tests.

Reference: category maps dataset.py:24-68, convert_to_simplified_category :70-74,
MisinformationDataset :132-178 (H5 per-sample groups; pre_embed keys), get_dataloader :181-192.
The H5 reader needs h5py (absent in this image): it is imported lazily and raises a clear error.
"""
from __future__ import annotations

import logging
import os

import numpy as np
import torch
from torch.utils.data import DataLoader, Dataset

logger = logging.getLogger(__name__)

category_to_labels = {
    "Support_Text": [0, 1, 1, 1],
    "Support_Multimodal": [0, 0, 0, 0],
    "Insufficient_Text": [1, 1, 1, 1],
    "Insufficient_Multimodal": [1, 1, 1, 0],
    "Refute": [2, 2, 2, 2],
}
labels_to_category = {tuple(v): k for k, v in category_to_labels.items()}
category_to_idx = {"Support_Text": 0, "Support_Multimodal": 1, "Insufficient_Text": 2,
                   "Insufficient_Multimodal": 3, "Refute": 4}
idx_to_category = {v: k for k, v in category_to_idx.items()}
simplified_category_mapping = {"Support_Text": "Support", "Support_Multimodal": "Support",
                               "Insufficient_Text": "NEI", "Insufficient_Multimodal": "NEI", "Refute": "Refute"}
simplified_category_to_idx = {"Support": 0, "NEI": 1, "Refute": 2}
simplified_idx_to_category = {v: k for k, v in simplified_category_to_idx.items()}

LABEL_TABLE = torch.tensor([category_to_labels[idx_to_category[i]] for i in range(5)], dtype=torch.int64)


def convert_to_simplified_category(category_idx):
    return simplified_category_to_idx[simplified_category_mapping[idx_to_category[category_idx]]]


def _store_paths(csv_path, pre_embed):
    """(h5 path, npz-directory path) the reference derives from the CSV path (dataset.py:136-138)"""
    base = os.path.splitext(csv_path)[0]
    h5 = base + "_embeddings.h5" if pre_embed else base + ".h5"
    return h5, os.path.splitext(h5)[0]


class MisinformationDataset(Dataset):
    """dataset.py:132-178: samples stored as groups str(idx) of `<csv base>.h5` (raw) or
    `<csv base>_embeddings.h5` (pre_embed). h5py is absent in this image, so the same groups are
    also read from a directory store `<csv base>[_embeddings]/<idx>.npz` (written by
    prepare_h5_dataset / mmfd.preembed.create_embeddings when h5py is missing). A missing raw store
    is built from the CSV (prepare_h5_dataset), as the reference does; a missing pre_embed store
    raises (preprocess_embeddings.py builds it)."""

    def __init__(self, csv_path, pre_embed=False):
        self.csv_path = csv_path
        self.pre_embed = pre_embed
        self.h5_path, self.npz_dir = _store_paths(csv_path, pre_embed)
        self.h5_file = None
        if not os.path.exists(self.h5_path) and not os.path.isdir(self.npz_dir):
            if pre_embed:
                raise FileNotFoundError(f"Pre-computed embeddings not found at {self.h5_path} (or {self.npz_dir}/). "
                                        "Run mmfd.preembed.create_embeddings first.")
            prepare_h5_dataset(csv_path, self.h5_path)
        if os.path.exists(self.h5_path):
            try:
                import h5py
            except ImportError as e:  # pragma: no cover - depends on the image
                raise ImportError(f"{self.h5_path} needs h5py") from e
            self.h5_file = h5py.File(self.h5_path, "r")
            self.length = len(self.h5_file.keys())
        else:
            self.length = len([f for f in os.listdir(self.npz_dir) if f.endswith(".npz")])

    def __len__(self):
        return self.length

    def _sample(self, idx):
        if self.h5_file is not None:
            return self.h5_file[str(idx)]
        return np.load(os.path.join(self.npz_dir, f"{idx}.npz"), allow_pickle=False)

    def __getitem__(self, idx):
        s = self._sample(idx)

        def txt(v):
            v = v[()]
            return v.decode() if isinstance(v, bytes) else str(v)

        if self.pre_embed:
            return {"id": str(idx), **{k: torch.from_numpy(np.asarray(s[k][()])) for k in
                                       ("claim_text_embeds", "doc_text_embeds", "claim_image_embeds",
                                        "doc_image_embeds", "labels")}}
        return {"id": str(idx), "claim": txt(s["claim"]), "claim_image": torch.from_numpy(np.asarray(s["claim_image"][()])),
                "document": txt(s["document"]), "document_image": torch.from_numpy(np.asarray(s["document_image"][()])),
                "labels": torch.from_numpy(np.asarray(s["labels"][()]))}

    def __del__(self):
        if getattr(self, "h5_file", None) is not None:
            self.h5_file.close()


def prepare_h5_dataset(csv_path, h5_path, enriched=False, device="cuda", batch_size=64):
    """dataset.py:76-129: one group per sample (claim, document, the two images through the
    Resize(256)+CenterCrop(256)+ToTensor+Normalize transform, the 4 path labels), samples whose
    claim or evidence image cannot be opened skipped. Images are decoded on the host and
    transformed on the GPU in batches (mmfd.preprocess "train", bit-exact with torchvision on PIL).
    Writes H5 when h5py is importable, else the directory store `<h5_path without .h5>/<idx>.npz`."""
    import pandas as pd
    from PIL import Image
    from .preprocess import ImagePreprocessor

    os.makedirs(os.path.dirname(os.path.abspath(h5_path)), exist_ok=True)
    cols = ["claim_enriched" if enriched else "claim", "claim_image", "evidence_enriched" if enriched else "evidence",
            "evidence_image", "category"]
    df = pd.read_csv(csv_path, index_col=0)[cols]
    try:
        import h5py
        out = h5py.File(h5_path, "w")
    except ImportError:
        out = None
        npz_dir = os.path.splitext(h5_path)[0]
        os.makedirs(npz_dir, exist_ok=True)
    pre = ImagePreprocessor("train", device=device)
    pending, valid = [], 0

    def flush():
        nonlocal valid
        if not pending:
            return
        px = pre([im for it in pending for im in (it[1], it[3])]).cpu().numpy()
        for j, (claim, _, doc, _, labels) in enumerate(pending):
            arrays = dict(claim=np.array(claim), document=np.array(doc), claim_image=px[2 * j],
                          document_image=px[2 * j + 1], labels=np.asarray(labels, np.int64))
            if out is not None:
                g = out.create_group(str(valid))
                for k, v in arrays.items():
                    g.create_dataset(k, data=v)
            else:
                np.savez(os.path.join(npz_dir, f"{valid}.npz"), **arrays)
            valid += 1
        pending.clear()

    for _, row in df.iterrows():
        try:
            ci = Image.open(row["claim_image"]).convert("RGB")
            di = Image.open(row["evidence_image"]).convert("RGB")
        except Exception as e:  # noqa: BLE001 - the reference skips any unreadable image (:102-110)
            logger.warning("Skipping sample due to missing image: %s", e)
            continue
        pending.append((str(row[cols[0]]), ci, str(row[cols[2]]), di,
                        category_to_labels.get(row["category"], [1, 1, 1, 1])))
        if len(pending) == batch_size:
            flush()
    flush()
    if out is not None:
        out.close()
    logger.info("Created dataset at %s with %d valid samples", h5_path, valid)
    return valid


class SyntheticFactifyDataset(Dataset):
    """Factify-shaped synthetic claim/evidence pairs (BASELINE §8d): token ids ~ U[1000, vocab) with
    [CLS]=101 / [SEP]=102, optional ragged lengths (0 = [PAD]), pixels ~ N(0, 1) (post-normalise
    distribution), labels drawn uniformly from the 5 category rows of category_to_labels.
    Items carry pre-tokenised texts (claim_input_ids / claim_attention_mask / document_...);
    `stack_pairs` collates them into FusionTrainer batches."""

    def __init__(self, n, seq_len=128, image_size=224, vocab_size=30522, seed=0, ragged=False):
        self.n, self.L, self.S, self.V, self.seed, self.ragged = n, seq_len, image_size, vocab_size, seed, ragged

    def __len__(self):
        return self.n

    def _ids(self, g):
        ids = torch.randint(1000, self.V, (self.L,), generator=g)
        ids[0] = 101
        n = int(torch.randint(16, self.L + 1, (1,), generator=g)) if self.ragged else self.L
        ids[n - 1] = 102
        mask = (torch.arange(self.L) < n).long()
        return ids * mask, mask

    def __getitem__(self, idx):
        g = torch.Generator().manual_seed(self.seed * 1000003 + idx)
        ci, cm = self._ids(g)
        di, dm = self._ids(g)
        cat = int(torch.randint(0, 5, (1,), generator=g))
        return {"id": str(idx), "claim_input_ids": ci, "claim_attention_mask": cm, "document_input_ids": di,
                "document_attention_mask": dm, "claim_image": torch.randn(3, self.S, self.S, generator=g),
                "document_image": torch.randn(3, self.S, self.S, generator=g), "labels": LABEL_TABLE[cat].clone()}


def synthetic_batch(B, seq_len=128, image_size=224, vocab_size=30522, seed=0, device="cuda", ragged=False):
    """A whole stacked batch generated on the device (bench inputs resident in HBM)."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    ids = torch.randint(1000, vocab_size, (2 * B, seq_len), generator=g)
    ids[:, 0] = 101
    if ragged:
        n = torch.randint(16, seq_len + 1, (2 * B,), generator=g)
    else:
        n = torch.full((2 * B,), seq_len)
    mask = (torch.arange(seq_len)[None] < n[:, None]).long()
    ids[torch.arange(2 * B), n - 1] = 102
    ids = ids * mask
    labels = LABEL_TABLE[torch.randint(0, 5, (B,), generator=g)]
    px = torch.randn(2 * B, 3, image_size, image_size, generator=g)
    return {"input_ids": ids.to(device), "attention_mask": mask.to(device), "pixel_values": px.to(device),
            "labels": labels.to(device)}


def stack_pairs(items, tokenizer=None, max_length=512):
    """collate_fn: dataset items -> one FusionTrainer batch.
      * pre_embed items (claim_text_embeds, ...): the four embedding tensors stacked + labels;
      * pre-tokenised items (SyntheticFactifyDataset): input_ids / attention_mask [2B, L] with the
        claims first, pixel_values [2B, 3, S, S] (claim images first), labels [B, 4];
      * raw items (MisinformationDataset: 'claim' / 'document' strings): tokenised with
        `tokenizer(..., truncation=True, padding=True, max_length=512)` as train.py:136,139 does
        (claims and documents padded to one common length here, as they share one encoder call)."""
    ids = [it["id"] for it in items]
    labels = torch.stack([torch.as_tensor(it["labels"]) for it in items])
    if "claim_text_embeds" in items[0]:
        out = {k: torch.stack([it[k] for it in items]) for k in
               ("claim_text_embeds", "doc_text_embeds", "claim_image_embeds", "doc_image_embeds")}
        return {"id": ids, **out, "labels": labels}
    px = torch.stack([it["claim_image"] for it in items] + [it["document_image"] for it in items])
    if "claim_input_ids" in items[0]:
        L = max(max(len(it["claim_input_ids"]), len(it["document_input_ids"])) for it in items)

        def pad(t):
            return torch.nn.functional.pad(torch.as_tensor(t), (0, L - len(t)))
        input_ids = torch.stack([pad(it["claim_input_ids"]) for it in items] + [pad(it["document_input_ids"]) for it in items])
        mask = torch.stack([pad(it["claim_attention_mask"]) for it in items] +
                           [pad(it["document_attention_mask"]) for it in items])
    else:
        if tokenizer is None:
            raise ValueError("raw text items need a tokenizer (no vocabulary ships offline: pass a local one)")
        enc = tokenizer([it["claim"] for it in items] + [it["document"] for it in items], truncation=True,
                        padding=True, return_tensors="pt", max_length=max_length)
        input_ids, mask = enc["input_ids"], enc["attention_mask"]
    return {"id": ids, "input_ids": input_ids, "attention_mask": mask, "pixel_values": px, "labels": labels}


def get_dataloader(csv_path, batch_size=32, num_workers=4, shuffle=False, pre_embed=False, collate_fn=None):
    """dataset.py:181-192 (plus an optional collate_fn, e.g. functools.partial(stack_pairs, tokenizer=...))"""
    return DataLoader(MisinformationDataset(csv_path, pre_embed=pre_embed), batch_size=batch_size, shuffle=shuffle,
                      num_workers=num_workers, pin_memory=True, collate_fn=collate_fn)
