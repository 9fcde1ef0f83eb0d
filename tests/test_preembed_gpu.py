"""Pre-embedding pass (preprocess_embeddings.py:11-116) on HIP encoders: every
sample's group holds the five datasets with the reference's shapes ([max_length, D_text] text
embeddings at max_length 512-style padding, [T, D_image] image embeddings, int64 labels), and
each stored embedding equals the encoder run on that sample alone (fp32, 1e-5 abs)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_create_embeddings_roundtrip(tmp_path):
    from mmfd.dataset import SyntheticFactifyDataset
    from mmfd.deberta import DebertaV2Config, DebertaV2Model
    from mmfd.encoders import ViTConfig, ViTModel
    from mmfd.preembed import KEYS, PreEmbedDataset, create_embeddings, embed_batch

    torch.manual_seed(0)
    deb = DebertaV2Model(DebertaV2Config(vocab_size=3000, hidden_size=64, num_hidden_layers=2, num_attention_heads=2,
                                         intermediate_size=128)).cuda().eval()
    vit = ViTModel(ViTConfig(image_size=32, patch_size=16, hidden_size=64, num_hidden_layers=2,
                             num_attention_heads=2, intermediate_size=128)).cuda().eval()
    ds = SyntheticFactifyDataset(5, seq_len=40, image_size=32, vocab_size=3000, seed=3, ragged=True)
    out = create_embeddings(ds, str(tmp_path / "emb"), deb, vit, batch_size=2, max_length=48, force_npz=True)
    rd = PreEmbedDataset(out)
    assert len(rd) == 5
    for i in (0, 3, 4):
        it = rd[i]
        assert set(KEYS) <= set(it) and it["id"] == str(i)
        assert it["claim_text_embeds"].shape == (48, 64) and it["doc_text_embeds"].shape == (48, 64)
        assert it["claim_image_embeds"].shape == (5, 64) and it["labels"].dtype == torch.int64
        s = ds[i]
        pad = lambda t: torch.nn.functional.pad(t, (0, 48 - t.numel()))[None].cuda()  # noqa: E731
        ct, dt, ci, di = embed_batch(deb, vit, pad(s["claim_input_ids"]), pad(s["claim_attention_mask"]),
                                     pad(s["document_input_ids"]), pad(s["document_attention_mask"]),
                                     s["claim_image"][None].cuda(), s["document_image"][None].cuda())
        for k, ref in zip(KEYS[:4], (ct, dt, ci, di)):
            assert (it[k] - ref[0].cpu()).abs().max().item() < 1e-5, k
        assert np.array_equal(it["labels"].numpy(), s["labels"].numpy())


def test_create_embeddings_with_swinv2(tmp_path):
    """the reference's own encoder pair (DeBERTa-v3 text, Swinv2 image; train.py:330-332) through
    create_embeddings: image groups hold the Swinv2 [tokens, features] last_hidden_state of the
    sample (here image 128 -> [64, 128]; swinv2-base at 256 gives the reference's [64, 1024])"""
    from mmfd.dataset import SyntheticFactifyDataset
    from mmfd.deberta import DebertaV2Config, DebertaV2Model
    from mmfd.preembed import PreEmbedDataset, create_embeddings
    from mmfd.swinv2 import Swinv2Config, Swinv2Model

    torch.manual_seed(1)
    deb = DebertaV2Model(DebertaV2Config(vocab_size=3000, hidden_size=64, num_hidden_layers=1, num_attention_heads=2,
                                         intermediate_size=128)).cuda().eval()
    swin = Swinv2Model(Swinv2Config(image_size=128, embed_dim=32, depths=(2, 2, 2), num_heads=(1, 2, 4),
                                    pretrained_window_sizes=(0, 0, 0))).cuda().eval()
    ds = SyntheticFactifyDataset(3, seq_len=24, image_size=128, vocab_size=3000, seed=5, ragged=True)
    out = create_embeddings(ds, str(tmp_path / "emb"), deb, swin, batch_size=2, max_length=32, force_npz=True)
    rd = PreEmbedDataset(out)
    assert len(rd) == 3
    for i in range(3):
        it = rd[i]
        assert it["claim_image_embeds"].shape == (64, 128) and it["doc_image_embeds"].shape == (64, 128)
        with torch.no_grad():
            ref = swin(ds[i]["claim_image"][None].cuda()).last_hidden_state[0].cpu()
        assert (it["claim_image_embeds"] - ref).abs().max().item() < 1e-5
