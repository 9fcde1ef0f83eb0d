"""CPU-only checks of the drop-in API surface and of the C-ABI library (loads, exports every
symbol include/mmfd.h declares; host-side hash matches the oracle). No GPU compute here."""
import json
import os
import re

import numpy as np
import pytest
import torch

import mmfd
from mmfd import kernels as K
from mmfd.model import MisinformationDetectionModel
from oracle.dropout_hash import dropout_hash, salt_of

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = os.path.join(ROOT, "tests", "golden")


def _header_symbols():
    src = open(os.path.join(ROOT, "include", "mmfd.h")).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w\*]+\s+\**(mmfd_\w+)\(", src, flags=re.M)))


def test_library_exports_every_declared_symbol():
    lib = K.load()
    syms = _header_symbols()
    assert len(syms) >= 25
    for s in syms:
        assert hasattr(lib, s), s
        assert s in K.SIGNATURES, f"{s} declared in include/mmfd.h but not bound in kernels.py"
    assert lib.mmfd_version() == K.ABI_VERSION == 3


def test_host_hash_matches_oracle():
    for seed, salt, idx in [(0, 0, 0), (1234, salt_of("x"), 17), (2 ** 40 + 5, 2 ** 63 + 11, 2 ** 35 + 3)]:
        assert K.dropout_hash(seed, salt, idx) == int(dropout_hash(seed, salt, np.array([idx], dtype=np.uint64))[0])
    assert K.salt_of("representation.text.self.attn") == salt_of("representation.text.self.attn")


def test_error_reporting_without_gpu_compute():
    # invalid arguments are rejected on the host before any launch
    a = K.GemmArgs()
    a.dtype = 7
    rc = K.lib().mmfd_gemm(a, None)
    assert rc != 0 and b"dtype" in K.lib().mmfd_last_error_string()


def test_struct_of_another_abi_layout_is_refused():
    """a caller built against another layout of mmfd_gemm_args / mmfd_attn_args
    (e.g. round 3's attention struct, 8 bytes shorter before drop_mask) passes another struct_size
    and is refused before any field is read, with a clear error string."""
    import ctypes
    lib = K.lib()
    a = K.GemmArgs()
    assert a.struct_size == ctypes.sizeof(K.GemmArgs)
    a.struct_size -= 8  # a shorter struct
    a.dtype = K.BF16
    assert lib.mmfd_gemm(a, None) == 1000  # MMFD_ERR_INVALID
    msg = lib.mmfd_last_error_string().decode()
    assert "struct_size" in msg and f"ABI version {K.ABI_VERSION}" in msg, msg
    assert lib.mmfd_gemm_workspace_bytes(a) == -1 and lib.mmfd_gemm_splits(a) == -1 and lib.mmfd_gemm_runs_split(a) == -1
    for fn in (lib.mmfd_attn_fwd, lib.mmfd_attn_bwd):
        t = K.AttnArgs()
        t.struct_size = ctypes.sizeof(K.AttnArgs) - 8
        assert fn(t, None) == 1000
        assert "mmfd_attn_args.struct_size" in lib.mmfd_last_error_string().decode()
    # the right size passes the guard (and then fails on its own argument checks, as before)
    b = K.GemmArgs()
    b.dtype = 7
    assert lib.mmfd_gemm(b, None) != 0 and b"bad dtype" in lib.mmfd_last_error_string()


@pytest.mark.parametrize("kw,fixture_key", [({}, "param_names"), ({"factify": True, "num_classes": 5}, "factify_param_names"),
                                             ({"text_only": True}, "text_only_param_names")])
def test_state_dict_names_match_reference(kw, fixture_key):
    z = np.load(os.path.join(G, "fusion_small.npz"), allow_pickle=False)
    ref = json.loads(str(z[fixture_key]))
    m = MisinformationDetectionModel(text_input_dim=48, image_input_dim=40, embed_dim=32, num_heads=4, dropout=0.0,
                                     hidden_dim=16, **kw)
    ours = [[k, list(v.shape)] for k, v in m.state_dict().items()]
    assert ours == ref


def test_full_dims_state_dict():
    z = np.load(os.path.join(G, "fusion_full.npz"), allow_pickle=False)
    ref = [(a, list(b)) for a, b in json.loads(str(z["param_names"]))]
    m = MisinformationDetectionModel(text_input_dim=768, image_input_dim=768)
    ours = [(k, list(v.shape)) for k, v in m.state_dict().items()]
    assert ours == ref and len(ours) == 108
    assert sum(p.numel() for p in m.parameters()) == 4410892


def test_reference_checkpoint_loads():
    """A reference `model_state_dict` (fixture: post-step params of the reference's train_epoch) loads."""
    z = np.load(os.path.join(G, "fusion_small.npz"), allow_pickle=False)
    sd = {k[5:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("post/")}
    m = MisinformationDetectionModel(text_input_dim=48, image_input_dim=40, embed_dim=32, num_heads=4, dropout=0.0,
                                     hidden_dim=16)
    m.load_state_dict(sd)


def test_forward_on_cpu_fails_loudly():
    m = MisinformationDetectionModel(text_input_dim=48, image_input_dim=40, embed_dim=32, num_heads=4, hidden_dim=16)
    with pytest.raises(RuntimeError):
        m(torch.randn(1, 3, 48), torch.randn(1, 3, 40), torch.randn(1, 3, 48), torch.randn(1, 3, 40))


def test_dropout_hash_statistics():
    """the one-round counter hash: keep rate within 3 sigma of 1-p over 2^20 consecutive indices,
    no correlation between neighbouring elements, different salts give independent masks"""
    from oracle.dropout_hash import keep_mask
    n = 1 << 20
    for p in (0.1, 0.5):
        k = keep_mask(1234, salt_of("stats"), (n,), p).astype(np.float64)
        sigma = (p * (1 - p) / n) ** 0.5
        assert abs(k.mean() - (1 - p)) < 3 * sigma
        c = np.corrcoef(k[:-1], k[1:])[0, 1]
        assert abs(c) < 5 / n ** 0.5
    a = keep_mask(7, salt_of("a"), (n,), 0.5).astype(np.float64)
    b = keep_mask(7, salt_of("b"), (n,), 0.5).astype(np.float64)
    assert abs(np.corrcoef(a, b)[0, 1]) < 5 / n ** 0.5


def test_deberta_host_buckets_and_names():
    """the product's host-side log buckets equal the oracle's torch restatement of
    make_log_bucket_position at every length up to 512, and DebertaV2Model carries the
    transformers DebertaV2Model state_dict names and shapes (a hub checkpoint loads unchanged)"""
    import numpy as np
    from transformers import DebertaV2Config as HC, DebertaV2Model as HM

    from mmfd.deberta import DebertaV2Config, DebertaV2Model, log_bucket_relative_positions
    from oracle.deberta import log_bucket_relative_positions as ref
    for L in (1, 7, 128, 300, 512):
        assert np.array_equal(log_bucket_relative_positions(L, 256, 512), ref(L, 256, 512))
    kw = dict(vocab_size=1000, hidden_size=64, num_hidden_layers=2, num_attention_heads=2, intermediate_size=128)
    ours = DebertaV2Model(DebertaV2Config(**kw)).state_dict()
    hf = HM(HC(max_position_embeddings=512, relative_attention=True, position_buckets=256, norm_rel_ebd="layer_norm",
               share_att_key=True, pos_att_type=["p2c", "c2p"], position_biased_input=False, type_vocab_size=0,
               **kw)).state_dict()
    assert {k: tuple(v.shape) for k, v in ours.items()} == {k: tuple(v.shape) for k, v in hf.items()}


def test_stepctx_derived_cache_tracks_weight_versions():
    """weight-derived tensors (packed biases, Swinv2 position-bias tables) persist across calls of a
    frozen encoder and are rebuilt after an in-place weight change; training contexts never cache"""
    import torch
    from mmfd import blocks as Bk

    w = torch.ones(4)
    store = {}
    calls = []

    def make():
        calls.append(1)
        return w * 2

    for _ in range(3):
        ctx = Bk.StepCtx({"w": w}, torch.float32, shadows=store)
        ctx.cache_derived = True
        t = ctx.derived("k", ["w"], make)
    assert len(calls) == 1 and torch.equal(t, torch.full((4,), 2.0))
    w.add_(1.0)
    ctx = Bk.StepCtx({"w": w}, torch.float32, shadows=store)
    ctx.cache_derived = True
    assert torch.equal(ctx.derived("k", ["w"], make), torch.full((4,), 4.0)) and len(calls) == 2
    ctx = Bk.StepCtx({"w": w}, torch.float32, shadows=store)      # cache_derived off (training)
    ctx.derived("k", ["w"], make)
    assert len(calls) == 3


def test_cached_weights_invalidate_on_load_state_dict_and_data_writes():
    """weight-derived caches (shadow_store) are dropped by load_state_dict, .to() and an
    explicit invalidate_caches() (writes through .data do not bump torch's version counter)."""
    from mmfd import blocks as Bk
    from mmfd.model import MisinformationDetectionModel

    m = MisinformationDetectionModel(text_input_dim=16, image_input_dim=16, embed_dim=8, num_heads=2, hidden_dim=4)
    st = Bk.shadow_store(m)
    st["k"] = (torch.zeros(1), [])
    st[("derived", "x")] = ((), torch.zeros(1))
    m.load_state_dict(m.state_dict())
    assert not Bk.shadow_store(m)
    st = Bk.shadow_store(m)
    st["k"] = (torch.zeros(1), [])
    with torch.no_grad():
        next(m.parameters()).data.copy_(torch.ones_like(next(m.parameters())))
    assert Bk.shadow_store(m)  # a .data write is invisible to version counters ...
    m.invalidate_caches()
    assert not Bk.shadow_store(m)  # ... hence the explicit call
    Bk.shadow_store(m)["k"] = (torch.zeros(1), [])
    m.float()
    assert not Bk.shadow_store(m)


def test_cli_flags_mirror_reference_defaults():
    """train.py:24-85: same flag names and defaults (mmfd's additions listed separately)."""
    from mmfd.train import parse_args
    a = parse_args([])
    want = dict(epochs=50, batch_size=32, lr=1e-4, num_workers=8, device=0, seed=42, embed_dim=256, num_heads=8,
                dropout=0.1, hidden_dim=64, num_classes=3, mlp_ratio=4.0, fused_attn=False,
                train_data="./data/preprocessed/train.csv", val_data=None, text_encoder="microsoft/deberta-v3-xsmall",
                output_dir="./results", save_every=2000, log_every=100, wandb_project="misinformation-detection",
                wandb_entity=None, freeze_text=False, freeze_image=False, validate_every_epoch=False, save_best=False,
                best_metric="avg_f1", log_confusion_matrix=False, log_confusion_matrix_every=1000, pre_embed=False,
                text_input_dim=384, image_input_dim=1024)
    for k, v in want.items():
        assert getattr(a, k) == v, k
    b = parse_args(["--pre_embed", "--freeze_text", "--text_input_dim", "768", "--save_every", "5"])
    assert b.pre_embed and b.freeze_text and not b.freeze_image and b.text_input_dim == 768 and b.save_every == 5


def test_stack_pairs_collates_every_item_kind():
    from mmfd.dataset import SyntheticFactifyDataset, stack_pairs
    ds = SyntheticFactifyDataset(3, seq_len=20, image_size=16, ragged=True)
    b = stack_pairs([ds[i] for i in range(3)])
    assert b["input_ids"].shape == (6, 20) and b["pixel_values"].shape == (6, 3, 16, 16) and b["labels"].shape == (3, 4)
    assert torch.equal(b["input_ids"][0], ds[0]["claim_input_ids"]) and torch.equal(b["input_ids"][3], ds[0]["document_input_ids"])
    emb = [{"id": str(i), "claim_text_embeds": torch.zeros(5, 4), "doc_text_embeds": torch.zeros(5, 4),
            "claim_image_embeds": torch.zeros(3, 6), "doc_image_embeds": torch.zeros(3, 6),
            "labels": torch.tensor([0, 1, 1, 1])} for i in range(2)]
    e = stack_pairs(emb)
    assert e["claim_text_embeds"].shape == (2, 5, 4) and e["labels"].shape == (2, 4)
    with pytest.raises(ValueError):
        stack_pairs([{"id": "0", "claim": "a", "document": "b", "claim_image": torch.zeros(3, 4, 4),
                      "document_image": torch.zeros(3, 4, 4), "labels": torch.zeros(4, dtype=torch.long)}])


def test_misinformation_dataset_reads_npz_store(tmp_path):
    import numpy as np
    from mmfd.dataset import MisinformationDataset, get_dataloader
    d = tmp_path / "train_embeddings"
    d.mkdir()
    for i in range(3):
        np.savez(d / f"{i}.npz", claim_text_embeds=np.full((4, 2), i, np.float32), doc_text_embeds=np.zeros((4, 2), np.float32),
                 claim_image_embeds=np.zeros((3, 5), np.float32), doc_image_embeds=np.zeros((3, 5), np.float32),
                 labels=np.array([0, 1, 1, 1]))
    ds = MisinformationDataset(str(tmp_path / "train.csv"), pre_embed=True)
    assert len(ds) == 3 and ds[2]["claim_text_embeds"][0, 0].item() == 2.0 and ds[1]["id"] == "1"
    assert next(iter(get_dataloader(str(tmp_path / "train.csv"), batch_size=3, num_workers=0, pre_embed=True)))["labels"].shape == (3, 4)
    with pytest.raises(FileNotFoundError):
        MisinformationDataset(str(tmp_path / "missing.csv"), pre_embed=True)


def test_custom_op_boundary_schemas_and_fake_kernels():
    """torch.ops.mmfd.* (libmmfd_torch.so over the C ABI): schemas declare their mutated outputs,
    and the fake kernels let the ops trace without a device (FakeTensorMode)."""
    from torch._subclasses.fake_tensor import FakeTensorMode
    K.load()
    ops = torch.ops.mmfd
    for name in ("gemm", "linear", "attn_fwd", "attn_bwd", "layernorm_fwd", "layernorm_bwd", "xent", "adamw",
                 "seq_mean_fwd", "seq_mean_bwd", "cast", "cosine_scores", "topk"):
        assert hasattr(ops, name), name
    sch = str(ops.gemm.default._schema)
    assert "Tensor(a!) out" in sch and "Tensor(b!)? aux" in sch and "Tensor(c!)? a_rowsum" in sch
    assert "Tensor(a!) out, Tensor(b!) lse" in str(ops.attn_fwd.default._schema)
    with FakeTensorMode():
        x = torch.empty(2, 5, 48, device="cuda")
        w = torch.empty(24, 48, device="cuda")
        assert ops.linear(x, w, None, 1).shape == (2, 5, 24)
        out = torch.empty(10, 24, device="cuda")
        ops.gemm(x.reshape(10, 48), w, False, False, out, 1.0, 0.0, None, None, False, 0, None, 0.0, None, 0, 0,
                 None, 0.0)


def test_checked_state_dict_load():
    """extractor / re-ranker checkpoints load strictly except for named benign keys
    (blocks.load_state_dict_checked): a mismatched checkpoint raises instead of leaving random
    weights behind plausible outputs"""
    import torch.nn as nn
    from mmfd.blocks import load_state_dict_checked
    m = nn.Sequential(nn.Linear(4, 3), nn.Linear(3, 2))
    sd = {k: v.clone() + 1 for k, v in m.state_dict().items()}
    load_state_dict_checked(m, dict(sd, **{"pooler.dense.weight": torch.zeros(2)}), benign=("pooler",))
    assert torch.equal(m[0].weight, sd["0.weight"])
    with pytest.raises(RuntimeError, match="unexpected"):
        load_state_dict_checked(m, dict(sd, extra=torch.zeros(1)))
    with pytest.raises(RuntimeError, match="missing"):
        load_state_dict_checked(m, {k: v for k, v in sd.items() if k != "1.bias"})


def _rewrite_pickle_module(raw: bytes, old: bytes, new: bytes) -> bytes:
    """the same torch.save archive with a pickle global's module path renamed (simulates a
    checkpoint written under numpy 1.x, whose scalars pickle as numpy.core.multiarray.scalar)"""
    import io
    import zipfile
    src, dst = zipfile.ZipFile(io.BytesIO(raw)), io.BytesIO()
    with zipfile.ZipFile(dst, "w", compression=zipfile.ZIP_STORED) as z:
        for info in src.infolist():
            data = src.read(info.filename)
            if info.filename.endswith("data.pkl"):
                assert old in data
                data = data.replace(old, new)
            z.writestr(info, data)
    return dst.getvalue()


@pytest.mark.parametrize("numpy1", [False, True])
def test_best_model_checkpoint_with_numpy_metric_loads(tmp_path, numpy1):
    """the reference's best_model.pt (train.py:413-428) holds the best metric as a numpy
    scalar (np.mean of F1s) next to model_state_dict / optimizer_state_dict; mmfd's weights-only
    loader (MisinformationPredictor, --init_checkpoint) must read it, and still refuse other globals."""
    import io

    from mmfd.train import load_checkpoint
    m = MisinformationDetectionModel(text_input_dim=48, image_input_dim=40, embed_dim=32, num_heads=4, hidden_dim=16)
    opt = torch.optim.AdamW(m.parameters(), lr=1e-4)
    ck = {"epoch": 3, "global_step": np.int64(1200), "model_state_dict": m.state_dict(),
          "optimizer_state_dict": opt.state_dict(), "avg_f1": np.mean(np.array([0.5, 0.7, 0.6]))}
    buf = io.BytesIO()
    torch.save(ck, buf)
    raw = buf.getvalue()
    if numpy1:
        raw = _rewrite_pickle_module(raw, b"numpy._core.multiarray", b"numpy.core.multiarray")
    path = tmp_path / "best_model.pt"
    path.write_bytes(raw)
    with pytest.raises(Exception):
        torch.load(path, map_location="cpu", weights_only=True)  # the plain loader refuses it
    got = load_checkpoint(path)
    assert float(got["avg_f1"]) == pytest.approx(0.6) and int(got["global_step"]) == 1200
    m2 = MisinformationDetectionModel(text_input_dim=48, image_input_dim=40, embed_dim=32, num_heads=4, hidden_dim=16)
    m2.load_state_dict(got["model_state_dict"])
    for k, v in m.state_dict().items():
        assert torch.equal(v, m2.state_dict()[k])
    bad = tmp_path / "bad.pt"  # any other global still refuses
    torch.save({"model_state_dict": m.state_dict(), "x": io.BytesIO}, bad)
    with pytest.raises(Exception):
        load_checkpoint(bad)


def test_stale_shadow_entries_expire_with_their_store():
    """blocks.SHADOW_OF entries whose module (shadow store) is gone are dropped by live_shadow, so a
    reused weight pointer is not treated as already shadowed"""
    import gc
    from mmfd import blocks as Bk

    class M:
        pass

    m = M()
    st = Bk.shadow_store(m)
    ptr = 0x7fff0000
    import weakref
    Bk.SHADOW_OF[ptr] = (None, (id(st), "w"), weakref.ref(st))
    Bk.SHADOW_OF[ptr + 64] = (None, (id(st), "w"), weakref.ref(st))
    assert Bk.live_shadow(ptr) is not None
    del m, st
    gc.collect()
    # the store's finalizer dropped both entries; a stale entry found later is dropped on lookup
    assert ptr not in Bk.SHADOW_OF and ptr + 64 not in Bk.SHADOW_OF
    dead = Bk._ShadowStore()
    Bk.SHADOW_OF[ptr] = (None, (id(dead), "w"), weakref.ref(dead))
    del dead
    assert Bk.live_shadow(ptr) is None and ptr not in Bk.SHADOW_OF


def test_gemm_g4_source_is_the_generator_output(tmp_path):
    """csrc/gemm_g4.hip is generated (tools/gen_gemm_g4.py): the committed file equals a fresh run"""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = tmp_path / "gemm_g4.hip"
    subprocess.run([sys.executable, os.path.join(root, "tools", "gen_gemm_g4.py")], check=True,
                   env={**os.environ, "G4_OUT": str(out)}, stdout=subprocess.DEVNULL)
    committed = os.path.join(root, "multimodal-misinformation-detection_amd", "csrc", "gemm_g4.hip")
    assert out.read_text() == open(committed).read()
