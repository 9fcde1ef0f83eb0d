"""Pre-embedding pass: `create_embeddings_h5` of
src/data_loader/preprocess_embeddings.py:11-116 on HIP encoders — claim and document texts through
the text encoder at max_length 512 (DeBERTa-v3, mmfd.deberta; :24-25, 63-80), both images through
the image encoder (:91-92), and per sample one group str(idx) holding claim_text_embeds,
doc_text_embeds, claim_image_embeds, doc_image_embeds and labels (:95-114) — the layout
MisinformationDataset(pre_embed=True) reads (dataset.py:132-178).

Differences: inputs are pre-tokenised (no tokenizer vocabulary offline; the items of
mmfd.dataset.SyntheticFactifyDataset have the keys used here); claim and document go through each
encoder as ONE stacked batch; the store is H5 when h5py is importable and otherwise a directory
with one `<idx>.npz` per sample holding the same datasets (h5py is absent in this image), read
back by `PreEmbedDataset`. The reference's image encoder, Swinv2-base-patch4-window8-256
([B,3,256,256] -> [B,64,1024]), is `mmfd.swinv2.Swinv2Model`; any mmfd image encoder with
`.last_hidden_state` (ViT-B/16) plugs in as well.
"""
from __future__ import annotations

import os

import numpy as np
import torch
from torch.utils.data import Dataset

KEYS = ("claim_text_embeds", "doc_text_embeds", "claim_image_embeds", "doc_image_embeds", "labels")


class EmbeddingWriter:
    """per-sample groups str(idx) (preprocess_embeddings.py:95-114): H5 if h5py is importable,
    else `<dir>/<idx>.npz`"""

    def __init__(self, path, force_npz=False):
        self.path = path
        self.h5 = None
        if not force_npz:
            try:
                import h5py
                self.h5 = h5py.File(path, "w")
            except ImportError:
                pass
        if self.h5 is None:
            os.makedirs(path, exist_ok=True)

    def write(self, idx, **arrays):
        if self.h5 is not None:
            g = self.h5.create_group(str(idx))
            for k, v in arrays.items():
                g.create_dataset(k, data=v)
        else:
            np.savez(os.path.join(self.path, f"{idx}.npz"), **arrays)

    def close(self):
        if self.h5 is not None:
            self.h5.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class PreEmbedDataset(Dataset):
    """the npz-directory store read back with MisinformationDataset(pre_embed=True)'s item dict"""

    def __init__(self, path):
        self.path = path
        self.n = len([f for f in os.listdir(path) if f.endswith(".npz")])

    def __len__(self):
        return self.n

    def __getitem__(self, idx):
        z = np.load(os.path.join(self.path, f"{idx}.npz"))
        return {"id": str(idx), **{k: torch.from_numpy(z[k]) for k in KEYS}}


@torch.no_grad()
def embed_batch(text_encoder, image_encoder, claim_ids, claim_mask, doc_ids, doc_mask, claim_images, doc_images):
    """(claim_text, doc_text, claim_image, doc_image) last_hidden_states of one batch; claim and
    document stacked through each encoder"""
    B = claim_ids.shape[0]
    T = text_encoder(input_ids=torch.cat([claim_ids, doc_ids]),
                     attention_mask=torch.cat([claim_mask, doc_mask])).last_hidden_state
    I = image_encoder(torch.cat([claim_images, doc_images])).last_hidden_state
    return T[:B], T[B:], I[:B], I[B:]


@torch.no_grad()
def create_embeddings(samples, out_path, text_encoder, image_encoder, batch_size=32, max_length=512,
                      device="cuda", force_npz=False):
    """preprocess_embeddings.py:11-116 over an indexable of pre-tokenised samples (keys
    claim_input_ids / claim_attention_mask / document_input_ids / document_attention_mask /
    claim_image / document_image / labels); texts padded or truncated to max_length (:63-76)."""
    text_encoder.eval()
    image_encoder.eval()

    def pad(t):
        t = torch.as_tensor(t)[:max_length]
        return torch.nn.functional.pad(t, (0, max_length - t.numel()))

    n = len(samples)
    with EmbeddingWriter(out_path, force_npz=force_npz) as w:
        for s0 in range(0, n, batch_size):
            items = [samples[i] for i in range(s0, min(n, s0 + batch_size))]
            st = lambda k, f=pad: torch.stack([f(it[k]) for it in items]).to(device)  # noqa: E731
            ct, dt_, ci, di = embed_batch(text_encoder, image_encoder, st("claim_input_ids"),
                                          st("claim_attention_mask"), st("document_input_ids"),
                                          st("document_attention_mask"), st("claim_image", torch.as_tensor),
                                          st("document_image", torch.as_tensor))
            assert ct.shape[1] == max_length and dt_.shape[1] == max_length  # :83-88
            ct, dt_, ci, di = (x.float().cpu().numpy() for x in (ct, dt_, ci, di))
            for j, it in enumerate(items):
                w.write(s0 + j, claim_text_embeds=ct[j], doc_text_embeds=dt_[j], claim_image_embeds=ci[j],
                        doc_image_embeds=di[j], labels=np.asarray(it["labels"]))
    return out_path
