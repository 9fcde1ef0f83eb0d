"""Pins the CPU oracle (oracle/) against fixtures produced by the reference code itself
(tests/golden/make_golden.py: the reference's src/model/model.py + train.train_epoch, and
transformers' BertModel / ViTModel). CPU only."""
import json
import os

import numpy as np
import pytest
import torch

from oracle import encoders as OE
from oracle import fusion_head as OF

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    return np.load(os.path.join(G, name), allow_pickle=False)


def _t(a):
    return torch.from_numpy(np.array(a))


def _params(z, prefix):
    return {k[len(prefix):]: _t(z[k]) for k in z.files if k.startswith(prefix)}


def _close(a, b, tol=2e-5):
    a, b = torch.as_tensor(a).double(), torch.as_tensor(b).double()
    assert a.shape == b.shape, (a.shape, b.shape)
    err = (a - b).abs().max().item()
    assert err <= tol * max(1.0, b.abs().max().item()), err


@pytest.fixture(scope="module")
def small():
    return _load("fusion_small.npz")


def test_fusion_small_eval_modes(small):
    z = small
    P = _params(z, "init/")
    X = {k: _t(z[k]) for k in ("X_t", "X_i", "E_t", "E_i")}
    with torch.no_grad():
        (a, b), (c, d) = OF.model_forward(P, X["X_t"], X["X_i"], X["E_t"], X["E_i"], num_heads=4)
        for n, y in zip(("tt", "ti", "it", "ii"), (a, b, c, d)):
            _close(y, z[f"eval_{n}"])
        _close(a, z["sdpa_tt"])  # SDPA branch == eager branch (layers.py:44-54)
        (u, n1), (n2, n3) = OF.model_forward(P, X_t=X["X_t"], E_t=X["E_t"], num_heads=4)
        assert n1 is None and n2 is None and n3 is None
        _close(u, z["uni_tt"])
        Pf = _params(z, "factify_init/")
        y, none = OF.model_forward(Pf, X["X_t"], X["X_i"], X["E_t"], X["E_i"], num_heads=4, factify=True)
        assert none is None
        _close(y, z["factify_out"])
        Pt = _params(z, "text_only_init/")
        y, _ = OF.model_forward(Pt, X_t=X["X_t"], E_t=X["E_t"], num_heads=4, text_only=True)
        _close(y, z["text_only_out"])


def test_fusion_small_train_step_matches_reference_train_epoch(small):
    """One step of train.py:123-188 (zero_grad, forward, sum of 4 CE, backward, AdamW lr=1e-4)."""
    z = small
    P = {k: v.clone().requires_grad_(True) for k, v in _params(z, "init/").items()}
    X = {k: _t(z[k]) for k in ("X_t", "X_i", "E_t", "E_i")}
    labels = _t(z["labels"])
    out = OF.model_forward(P, X["X_t"], X["X_i"], X["E_t"], X["E_i"], num_heads=4)
    total, per = OF.path_loss(out, labels)
    _close(total, z["train_total_loss"])
    for n, l in zip(("text_text", "text_image", "image_text", "image_image"), per):
        _close(l, z[f"train_loss_{n}"])
    total.backward()
    names = [k for k, _ in json.loads(str(z["param_names"]))]
    for k in names:
        gk = "grad/" + k
        if gk in z.files:
            _close(P[k].grad, z[gk], 5e-5)
        else:
            assert P[k].grad is None, f"{k} should get no gradient (unused LayerNorm)"
    assert sum("grad/" + k in z.files for k in names) == len(names) - 4  # text/image_self_ln2 w+b
    opt = torch.optim.AdamW([P[k] for k in names], lr=1e-4)
    opt.step()
    for k in names:
        _close(P[k].detach(), z["post/" + k], 1e-6)


def test_fusion_full_dims_recipe():
    z = _load("fusion_full.npz")
    names = json.loads(str(z["param_names"]))
    assert len(names) == 108  # the reference's 4-path state_dict
    P = OF.init_params_like_reference(names, int(z["seed"]))
    assert sum(v.numel() for v in P.values()) == int(z["n_params"]) == 4410892
    with torch.no_grad():
        (a, b), (c, d) = OF.model_forward(P, *(_t(z[k]) for k in ("X_t", "X_i", "E_t", "E_i")), num_heads=8)
    for y, k in zip((a, b, c, d), ("tt", "ti", "it", "ii")):
        _close(y, z[k], 1e-5)


def test_bert_small():
    z = _load("bert_small.npz")
    cfg = json.loads(str(z["config"]))
    P = {k: v.clone().requires_grad_(True) for k, v in _params(z, "param/").items()}
    out = OE.bert_forward(P, _t(z["input_ids"]), _t(z["attention_mask"]), _t(z["token_type_ids"]),
                          num_layers=cfg["num_hidden_layers"], num_heads=cfg["num_attention_heads"])
    _close(out, z["out"], 2e-5)
    (out * _t(z["R"])).sum().backward()
    for k in P:
        _close(P[k].grad, z["grad/" + k], 5e-5)


def test_vit_small():
    z = _load("vit_small.npz")
    cfg = json.loads(str(z["config"]))
    P = {k: v.clone().requires_grad_(True) for k, v in _params(z, "param/").items()}
    out = OE.vit_forward(P, _t(z["pixel_values"]), num_layers=cfg["num_hidden_layers"],
                         num_heads=cfg["num_attention_heads"], patch=cfg["patch_size"])
    _close(out, z["out"], 2e-5)
    (out * _t(z["R"])).sum().backward()
    for k in P:
        _close(P[k].grad, z["grad/" + k], 5e-5)


def test_bert_vit_base_recipe():
    z = _load("bert_base.npz")
    P = OF.init_params_like_reference(json.loads(str(z["param_names"])), int(z["seed"]))
    with torch.no_grad():
        out = OE.bert_forward(P, _t(z["input_ids"]), _t(z["attention_mask"]), num_layers=12, num_heads=12)
    _close(out, z["out"], 5e-5)
    z = _load("vit_base.npz")
    P = OF.init_params_like_reference(json.loads(str(z["param_names"])), int(z["seed"]))
    with torch.no_grad():
        out = OE.vit_forward(P, _t(z["pixel_values"]).float(), num_layers=12, num_heads=12)
    _close(out, z["out"], 5e-5)


# ---- evidence extractors (a12 ResNet50, a13 MPNet) ----------------------------------------------
def test_oracle_resnet_matches_transformers_fixture():
    from oracle.resnet import resnet_forward
    z = _load("resnet_small.npz")
    out = resnet_forward(_params(z, "param/"), _t(z["pixel_values"]), depths=tuple(z["depths"].tolist()))
    _close(out, z["out"])


def test_oracle_mpnet_matches_transformers_fixture():
    z = _load("mpnet_small.npz")
    cfg = json.loads(str(z["config"]))
    out = OE.mpnet_forward(_params(z, "param/"), _t(z["input_ids"]), _t(z["attention_mask"]),
                           num_layers=cfg["num_hidden_layers"], num_heads=cfg["num_attention_heads"],
                           eps=cfg["layer_norm_eps"])
    _close(out, z["out"])


def test_mpnet_buckets_product_host_code_matches_oracle():
    """the product computes the bucket map on the host once per length; it must equal HF's"""
    from mmfd.encoders import mpnet_relative_buckets
    for L in (1, 7, 40, 128, 300, 512):
        assert torch.equal(mpnet_relative_buckets(L).long(), OE.mpnet_buckets(L))


def test_extractor_state_dict_names():
    from mmfd.encoders import MPNetConfig, MPNetModel
    from mmfd.evidence import ResNet, resnet50
    z = _load("resnet_small.npz")
    mine = {k: tuple(v.shape) for k, v in ResNet((1, 1, 2, 1), 8).state_dict().items()
            if "num_batches" not in k and not k.startswith("fc.")}
    ref = {k[len("param/"):]: tuple(z[k].shape) for k in z.files if k.startswith("param/")}
    assert mine == ref
    assert sum(p.numel() for p in resnet50().parameters()) == 25_557_032  # torchvision resnet50
    zm = _load("mpnet_small.npz")
    cfg = json.loads(str(zm["config"]))
    m = MPNetModel(MPNetConfig(vocab_size=cfg["vocab_size"], hidden_size=cfg["hidden_size"],
                               num_hidden_layers=cfg["num_hidden_layers"], num_attention_heads=cfg["num_attention_heads"],
                               intermediate_size=cfg["intermediate_size"],
                               max_position_embeddings=cfg["max_position_embeddings"]))
    mine = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    ref = {k[len("param/"):]: tuple(zm[k].shape) for k in zm.files if k.startswith("param/")}
    ref.pop("embeddings.position_ids", None)
    assert mine == ref


# ---- retrieval scoring (§8(f) row 2) -----------------------------------------------------------------
def test_oracle_retrieval_cosine_matches_torch_modules():
    """oracle/retrieval.py restates nn.CosineSimilarity(dim=1, eps=1e-6) (the module
    im2im_retrieval.py:40 calls per corpus image) and util.cos_sim's F.normalize(eps=1e-12) form;
    pinned here against torch's own CPU implementations of both."""
    from oracle.retrieval import cosine_normalized, cosine_pair
    g = torch.Generator().manual_seed(3)
    q = torch.randn(3, 64, generator=g)
    c = torch.randn(50, 64, generator=g)
    c[7] = 0.0  # zero row: the eps clamp decides
    cos = torch.nn.CosineSimilarity(dim=1, eps=1e-6)
    ref = torch.stack([torch.stack([cos(q[i:i + 1].double(), c[j:j + 1].double())[0] for j in range(50)]) for i in range(3)])
    np.testing.assert_allclose(cosine_pair(q.numpy(), c.numpy()), ref.numpy(), rtol=1e-12, atol=1e-12)
    fn = torch.nn.functional.normalize
    ref2 = fn(q.double(), p=2, dim=1) @ fn(c.double(), p=2, dim=1).T
    np.testing.assert_allclose(cosine_normalized(q.numpy(), c.numpy()), ref2.numpy(), rtol=1e-12, atol=1e-12)


def test_oracle_retrieval_order_and_distinct_filter():
    """sorted(..., key=score, reverse=True) keeps corpus order among equal scores, and the
    reference's filter keeps the first entry of every distinct score (im2im_retrieval.py:94-106)"""
    from oracle.retrieval import ranked, retrieve_unique
    s = np.array([0.5, 0.9, 0.5, 0.9, 0.1, 0.7, 0.9])
    items = sorted({i: float(v) for i, v in enumerate(s)}.items(), key=lambda x: x[1], reverse=True)
    assert [i for i, _ in items] == list(ranked(s))
    assert retrieve_unique(s, 3) == [(1, 0.9), (5, 0.7), (0, 0.5)]
    assert retrieve_unique(s, 10) == [(1, 0.9), (5, 0.7), (0, 0.5), (4, 0.1)]


# ---- raw-image preprocessing (§8(f) row 3) ------------------------------------------------------------
def _resample_with_taps(a, oh, ow):
    """PIL's two-pass 8-bit integer resample driven by mmfd.preprocess.pil_taps (host logic under
    test: the taps the GPU kernels consume)"""
    from mmfd.preprocess import pil_taps
    tx, ty = pil_taps(a.shape[1], ow).astype(np.int64), pil_taps(a.shape[0], oh).astype(np.int64)
    tmp = np.zeros((a.shape[0], ow, 3), np.int64)
    for xx in range(ow):
        x0, n = tx[xx, 0], tx[xx, 1]
        s = (1 << 21) + (a[:, x0:x0 + n, :].astype(np.int64) * tx[xx, 2:2 + n][None, :, None]).sum(1)
        tmp[:, xx] = np.clip(s >> 22, 0, 255)
    out = np.zeros((oh, ow, 3), np.int64)
    for yy in range(oh):
        y0, n = ty[yy, 0], ty[yy, 1]
        s = (1 << 21) + (tmp[y0:y0 + n] * ty[yy, 2:2 + n][:, None, None]).sum(0)
        out[yy] = np.clip(s >> 22, 0, 255)
    return out.astype(np.uint8)


@pytest.mark.parametrize("h,w,oh,ow", [(375, 500, 256, 341), (480, 640, 224, 224), (100, 90, 224, 224),
                                       (256, 300, 256, 300), (257, 1000, 224, 224), (31, 7, 256, 57)])
def test_pil_taps_reproduce_pil_resize_exactly(h, w, oh, ow):
    from PIL import Image
    a = np.random.default_rng(h * w).integers(0, 256, (h, w, 3), dtype=np.uint8)
    ref = np.asarray(Image.fromarray(a).resize((ow, oh), Image.BILINEAR))
    assert np.array_equal(_resample_with_taps(a, oh, ow), ref)


def test_preprocess_oracle_matches_torch_tensor_ops_and_size_rules():
    """oracle/preprocess.py's ToTensor/Normalize arithmetic equals torch's fp32 CPU ops bit for bit;
    the torchvision size / crop rules (Resize(int) keeps the aspect ratio with a truncated long
    side, CenterCrop rounds the origin with Python's round) on known cases"""
    from PIL import Image
    from oracle.preprocess import preprocess, resized_size
    from mmfd.preprocess import center_crop_origin, resized_size as host_size
    assert resized_size(375, 500, 256) == (256, 341) and resized_size(500, 375, 256) == (341, 256)
    assert resized_size(256, 999, 256) == (256, 999) and resized_size(10, 20, (224, 224)) == (224, 224)
    for hw in [(375, 500), (500, 375), (256, 257), (100, 90), (999, 256)]:
        assert host_size(*hw, 256) == resized_size(*hw, 256)
    assert center_crop_origin(256, 341, 256) == (0, 42) and center_crop_origin(257, 256, 256) == (0, 0)
    a = np.random.default_rng(1).integers(0, 256, (300, 400, 3), dtype=np.uint8)
    got = preprocess(Image.fromarray(a), (224, 224), None, (0.485, 0.456, 0.406), (0.229, 0.224, 0.225))
    img = np.asarray(Image.fromarray(a).resize((224, 224), Image.BILINEAR))
    t = torch.from_numpy(img.copy()).permute(2, 0, 1).contiguous().to(torch.float32).div(255)
    t = t.sub_(torch.tensor([0.485, 0.456, 0.406])[:, None, None]).div_(torch.tensor([0.229, 0.224, 0.225])[:, None, None])
    assert np.array_equal(got, t.numpy())


def test_deberta_oracle_matches_transformers_fixture():
    """oracle/deberta.py (DeBERTa-v3, the reference's default text encoder) against transformers'
    DebertaV2Model output in tests/golden/deberta_small.npz (L=300 with a padded row)."""
    from oracle.deberta import deberta_forward
    z = np.load(os.path.join(G, "deberta_small.npz"))
    P = {k[2:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("w.")}
    out = deberta_forward(P, torch.from_numpy(z["input_ids"]), torch.from_numpy(z["attention_mask"]),
                          num_layers=2, num_heads=2)
    assert (out - torch.from_numpy(z["last_hidden_state"])).abs().max().item() < 1e-5


def test_deberta_log_buckets():
    """make_log_bucket_position: identity inside +-mid, odd-symmetric, within +-(S-1) up to L=512"""
    from oracle.deberta import log_bucket_relative_positions
    r = log_bucket_relative_positions(512, 256, 512)
    assert (r == -r.T).all()
    assert r[200, 100] == 100 and r[0, 127] == -127
    assert np.abs(r).max() <= 255


SWIN_SMALL = dict(image_size=128, patch_size=4, num_channels=3, embed_dim=32, depths=(2, 2, 2), num_heads=(1, 2, 4),
                  window_size=8, mlp_ratio=4.0, layer_norm_eps=1e-5, pretrained_window_sizes=(0, 0, 0))


def test_swinv2_oracle_matches_transformers_fixture():
    """oracle/swinv2.py (Swinv2, the reference's default image encoder) against transformers'
    Swinv2Model in tests/golden/swinv2_small.npz (shifted windows in stages 1-2, one head's
    logit_scale above the ln(100) clamp): last_hidden_state and pooler_output."""
    from oracle.swinv2 import swinv2_forward
    z = np.load(os.path.join(G, "swinv2_small.npz"))
    P = {k[2:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("w.")}
    out, pooled = swinv2_forward(P, torch.from_numpy(z["pixel_values"]), SWIN_SMALL)
    assert (out - torch.from_numpy(z["last_hidden_state"])).abs().max().item() < 1e-5
    assert (pooled - torch.from_numpy(z["pooler_output"])).abs().max().item() < 1e-5


@pytest.mark.parametrize("R,ws,shift", [(64, 8, 0), (64, 8, 4), (32, 8, 4), (8, 8, 0)])
def test_swinv2_host_geometry_matches_oracle(R, ws, shift):
    """the product's host-side tables (mmfd.swinv2: window order as one row permutation, shift mask,
    coords table / relative position index) equal the oracle's roll + window_partition / mask /
    create_coords_table_and_index"""
    import mmfd.swinv2 as S
    from oracle import swinv2 as O
    nat = torch.arange(R * R, dtype=torch.float32).view(1, R, R, 1)
    rolled = torch.roll(nat, shifts=(-shift, -shift), dims=(1, 2)) if shift else nat
    want = O._partition(rolled, ws).reshape(-1).long().numpy()
    assert np.array_equal(S.window_order(R, ws, shift), want)
    if shift:
        assert np.array_equal(S.shift_mask(R, ws, shift), O._mask(R, R, ws, shift).numpy())
    t, rpi = S.coords_table_and_index(ws)
    t2, rpi2 = O._coords(ws, 0)
    assert torch.equal(t, t2.float()) and torch.equal(rpi.long(), rpi2.reshape(-1))


def test_cross_encoder_oracle_matches_transformers_fixture():
    """oracle.encoders.cross_encoder_forward vs transformers BertForSequenceClassification
    (num_labels 1, the ms-marco-MiniLM-L-6-v2 architecture scaled down)."""
    z = _load("cross_encoder_small.npz")
    cfg = json.loads(str(z["config"]))
    P = _params(z, "param/")
    args = (_t(z["input_ids"]), _t(z["attention_mask"]), _t(z["token_type_ids"]))
    kw = dict(num_layers=cfg["num_hidden_layers"], num_heads=cfg["num_attention_heads"])
    _close(OE.cross_encoder_forward(P, *args, activation=None, **kw), z["logits"], 2e-5)
    _close(OE.cross_encoder_forward(P, *args, **kw), z["scores"], 2e-5)
