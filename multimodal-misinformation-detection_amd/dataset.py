"""Mirror of src/model/dataset.py: label maps, Dataset / DataLoader factory (same dict keys), plus a
synthetic Factify-shaped pair generator for benchmarks and tests.

Reference: category maps dataset.py:24-68, convert_to_simplified_category :70-74,
MisinformationDataset :132-178 (H5 per-sample groups; pre_embed keys), get_dataloader :181-192.
The H5 reader needs h5py (absent in this image): it is imported lazily and raises a clear error.
"""
from __future__ import annotations

import os

import torch
from torch.utils.data import DataLoader, Dataset

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


class MisinformationDataset(Dataset):
    """dataset.py:132-178: samples stored as H5 groups str(idx) (needs h5py)."""

    def __init__(self, csv_path, pre_embed=False):
        self.csv_path = csv_path
        self.pre_embed = pre_embed
        base = os.path.splitext(csv_path)[0]
        self.h5_path = base + "_embeddings.h5" if pre_embed else base + ".h5"
        try:
            import h5py
        except ImportError as e:  # pragma: no cover - depends on the image
            raise ImportError("MisinformationDataset reads the reference's H5 files and needs h5py") from e
        if not os.path.exists(self.h5_path):
            raise FileNotFoundError(f"{self.h5_path} not found (build it with the reference's preprocessing)")
        self.h5_file = h5py.File(self.h5_path, "r")
        self.length = len(self.h5_file.keys())

    def __len__(self):
        return self.length

    def __getitem__(self, idx):
        s = self.h5_file[str(idx)]
        if self.pre_embed:
            return {"id": str(idx), **{k: torch.from_numpy(s[k][()]) for k in
                                       ("claim_text_embeds", "doc_text_embeds", "claim_image_embeds",
                                        "doc_image_embeds", "labels")}}
        return {"id": str(idx), "claim": s["claim"][()].decode(), "claim_image": torch.from_numpy(s["claim_image"][()]),
                "document": s["document"][()].decode(), "document_image": torch.from_numpy(s["document_image"][()]),
                "labels": torch.from_numpy(s["labels"][()])}


class SyntheticFactifyDataset(Dataset):
    """Factify-shaped synthetic claim/evidence pairs (BASELINE §8d): token ids ~ U[1000, vocab) with
    [CLS]=101 / [SEP]=102, optional ragged lengths (0 = [PAD]), pixels ~ N(0, 1) (post-normalise
    distribution), labels drawn uniformly from the 5 category rows of category_to_labels.
    Items use the pre-tokenised keys of the mmfd train step (see train.stack_pairs)."""

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


def get_dataloader(csv_path, batch_size=32, num_workers=4, shuffle=False, pre_embed=False):
    """dataset.py:181-192"""
    return DataLoader(MisinformationDataset(csv_path, pre_embed=pre_embed), batch_size=batch_size, shuffle=shuffle,
                      num_workers=num_workers, pin_memory=True)
