"""Evidence-corpus extractors (SURVEY §8 a12 ResNet50, a13 MPNet) on the HIP path vs the
transformers-generated fixtures and the CPU oracle.

Tolerances: fp32 — max abs error 1e-4 relative to the output's max magnitude (1e-3 at full
ResNet50 depth, where 53 folded-BN convolutions accumulate rounding); bf16 — 5e-2 relative
(bf16 activations between layers, fp32 accumulation). Conv kernels (im2col, max/avg pool) are
bit-exact data movement / fp32 reductions checked against torch.
"""
import io
import json
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

import mmfd
from mmfd import kernels as K
from mmfd.encoders import MPNetConfig, MPNetModel
from mmfd.evidence import ImageCorpus, ImageSimilarity, ResNet, SentenceEncoder, resnet50
from oracle import encoders as OE
from oracle.resnet import resnet_forward

pytestmark = pytest.mark.gpu
DEV = "cuda"
G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    return np.load(os.path.join(G, name), allow_pickle=False)


def _rel(got, ref):
    got, ref = torch.as_tensor(got).double().cpu(), torch.as_tensor(ref).double().cpu()
    assert got.shape == ref.shape, (got.shape, ref.shape)
    return (got - ref).abs().max().item() / max(ref.abs().max().item(), 1e-6)


def _resnet_from_fixture(z, precision):
    m = ResNet(tuple(z["depths"].tolist()), int(z["width"]))
    sd = {k[len("param/"):]: torch.from_numpy(np.array(z[k])) for k in z.files if k.startswith("param/")}
    m.load_state_dict(sd, strict=False)
    return m.to(DEV).set_precision(precision)


# ---- kernels --------------------------------------------------------------------------------------
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("k,stride,pad", [(3, 1, 1), (3, 2, 1), (1, 2, 0), (7, 2, 3)])
def test_im2col_nhwc_exact(dtype, k, stride, pad):
    N, H, W, C = 2, 9, 11, 16
    x = torch.randn(N, H, W, C).to(dtype)
    cols, Ho, Wo = K.im2col_nhwc(x.to(DEV).view(N * H * W, C), N, H, W, C, k, stride, pad, Kpad=k * k * C + 8)
    ref = F.unfold(x.permute(0, 3, 1, 2).float(), k, padding=pad, stride=stride)  # [N, C*k*k, L], (c, kh, kw)
    ref = ref.view(N, C, k, k, -1).permute(0, 4, 2, 3, 1).reshape(N * Ho * Wo, k * k * C)
    got = cols.float().cpu()
    assert torch.equal(got[:, :k * k * C], ref.to(dtype).float())
    assert torch.count_nonzero(got[:, k * k * C:]) == 0


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_stem_im2col_maxpool_avgpool(dtype):
    x = torch.randn(2, 3, 20, 18)
    cols, Ho, Wo = K.im2col_nchw(x.to(DEV), 7, 2, 3, 152, dtype)
    ref = F.unfold(x, 7, padding=3, stride=2).view(2, 3, 7, 7, -1).permute(0, 4, 2, 3, 1).reshape(2 * Ho * Wo, 147)
    assert torch.equal(cols.float().cpu()[:, :147], ref.to(dtype).float())
    y = torch.randn(2, 10, 9, 32).to(dtype)
    mp, Ho, Wo = K.maxpool_nhwc(y.to(DEV).view(-1, 32), 2, 10, 9, 32)
    ref = F.max_pool2d(y.float().permute(0, 3, 1, 2), 3, 2, 1).permute(0, 2, 3, 1).reshape(-1, 32)
    assert torch.equal(mp.float().cpu(), ref)
    ap = K.global_avgpool(y.to(DEV).view(-1, 32), 2, 90, 32)
    assert (ap.cpu() - y.float().mean((1, 2))).abs().max().item() < 1e-5


# ---- ResNet (a12) -----------------------------------------------------------------------------------
def test_resnet_small_matches_fixture_fp32():
    z = _load("resnet_small.npz")
    m = _resnet_from_fixture(z, "fp32")
    out = m(torch.from_numpy(z["pixel_values"]).to(DEV))
    torch.cuda.synchronize()
    assert _rel(out, z["out"]) < 1e-4


def test_resnet_small_bf16_close():
    z = _load("resnet_small.npz")
    m = _resnet_from_fixture(z, "bf16")
    out = m(torch.from_numpy(z["pixel_values"]).to(DEV))
    assert _rel(out, z["out"]) < 5e-2


def test_resnet50_full_vs_oracle():
    """full resnet50 at 224x224 (random init, non-trivial BN statistics) vs the CPU oracle"""
    torch.manual_seed(0)
    m = resnet50()
    g = torch.Generator().manual_seed(1)
    with torch.no_grad():
        for mod in m.modules():
            if isinstance(mod, torch.nn.BatchNorm2d):
                mod.running_mean.copy_(torch.randn(mod.running_mean.shape, generator=g) * 0.1)
                mod.running_var.copy_(torch.rand(mod.running_var.shape, generator=g) + 0.5)
                mod.weight.copy_(torch.rand(mod.weight.shape, generator=g) * 0.5 + 0.5)
    P = {k: v.clone() for k, v in m.state_dict().items()}
    x = torch.randn(2, 3, 224, 224, generator=g)
    ref = resnet_forward(P, x)
    m = m.to(DEV)
    out = m.set_precision("fp32")(x.to(DEV))
    assert _rel(out, ref) < 1e-3
    outb = m.set_precision("bf16")(x.to(DEV))
    assert _rel(outb, ref) < 5e-2


def test_image_similarity_and_corpus(tmp_path):
    from PIL import Image
    rng = np.random.default_rng(0)
    for i in range(5):
        Image.fromarray(rng.integers(0, 255, (40 + i, 50, 3), dtype=np.uint8)).save(tmp_path / f"img{i}.png")
    (tmp_path / "notes.txt").write_text("skip me")
    ext = ImageSimilarity(model=ResNet((1, 1, 1, 1), 8), precision="fp32")
    f = ext.extract_features(str(tmp_path / "img0.png"))
    assert f.shape == (256,) and f.device.type == "cpu"
    buf = io.BytesIO()
    Image.open(tmp_path / "img0.png").save(buf, format="PNG")
    buf.seek(0)
    assert torch.allclose(ext.extract_features(buf), f)
    assert abs(ImageSimilarity.similarity(f, f) - 1.0) < 1e-9
    for name in ("feats.npz", "feats.pkl"):  # .npz archive / the reference's pickle
        corpus = ImageCorpus(str(tmp_path / name), extractor=ext, batch_size=2)
        corpus.create_feature_corpus(str(tmp_path))
        assert len(corpus.feature_dict) == 5
        again = ImageCorpus(str(tmp_path / name), extractor=ext)
        assert set(again.feature_dict) == set(corpus.feature_dict)
        p0 = str(tmp_path / "img0.png")
        assert torch.allclose(again.feature_dict[p0], f, atol=1e-5)
    # batched and single extraction agree
    from oracle.preprocess import preprocess
    from mmfd.preprocess import MODES
    c = MODES["retrieval"]
    batch = torch.stack([torch.from_numpy(preprocess(Image.open(tmp_path / f"img{i}.png"), c["resize"], None, c["mean"],
                                                     c["std"])) for i in range(5)])
    fb = ext.extract_batch(batch).cpu()
    assert (fb[0] - f).abs().max().item() < 1e-4


def test_corpus_pinned_ring_equals_thread_decode(tmp_path):
    """config 5 host path: the corpus build that decodes in worker processes
    straight into the page-locked shared ring (mmfd.hostdecode.PinnedDecodeRing: asynchronous
    uploads, device-side preprocessing from the uploaded pixels, features kept on the device until
    the end) gives bit-identical features to the round-3 thread-pool decode + host staging; a ring
    with a small per-image space sends the larger images through the overflow path."""
    from PIL import Image

    from mmfd.hostdecode import PinnedDecodeRing
    rng = np.random.default_rng(3)
    d = tmp_path / "imgs"
    d.mkdir()
    for i in range(23):  # mixed sizes and formats, three batches of 8 (the last ragged)
        h, w = 60 + 13 * (i % 7), 80 + 11 * (i % 5)
        im = Image.fromarray(rng.integers(0, 255, (h, w, 3), dtype=np.uint8))
        im.save(d / f"x{i:02d}.{'png' if i % 3 == 0 else 'jpg'}")
    ext = ImageSimilarity(model=ResNet((1, 1, 1, 1), 8), precision="fp32")
    thr = ImageCorpus(str(tmp_path / "t.pkl"), extractor=ext, batch_size=8, decode_workers=3, decode="threads")
    thr.create_feature_corpus(str(d))
    for cap in (1 << 20, 4 * 4096):  # roomy / most images overflow their group's space
        ring = ImageCorpus(str(tmp_path / f"r{cap}.pkl"), extractor=ext, batch_size=8, decode_workers=3)
        ring._ring = PinnedDecodeRing(8, DEV, workers=3, group=3, cap=cap)
        try:
            ring.create_feature_corpus(str(d))
        finally:
            ring.close()
        assert list(ring.feature_dict) == list(thr.feature_dict)
        for k in thr.feature_dict:
            assert torch.equal(ring.feature_dict[k], thr.feature_dict[k]), (cap, k)


# ---- MPNet (a13) ------------------------------------------------------------------------------------
def _mpnet_from_fixture(z, precision):
    cfg = json.loads(str(z["config"]))
    m = MPNetModel(MPNetConfig(vocab_size=cfg["vocab_size"], hidden_size=cfg["hidden_size"],
                               num_hidden_layers=cfg["num_hidden_layers"], num_attention_heads=cfg["num_attention_heads"],
                               intermediate_size=cfg["intermediate_size"],
                               max_position_embeddings=cfg["max_position_embeddings"],
                               layer_norm_eps=cfg["layer_norm_eps"]))
    sd = {k[len("param/"):]: torch.from_numpy(np.array(z[k])) for k in z.files if k.startswith("param/")}
    sd.pop("embeddings.position_ids", None)
    m.load_state_dict(sd)
    return m.to(DEV).set_precision(precision)


@pytest.mark.parametrize("precision,tol", [("fp32", 1e-4), ("bf16", 5e-2)])
def test_mpnet_small_matches_fixture(precision, tol):
    z = _load("mpnet_small.npz")
    m = _mpnet_from_fixture(z, precision)
    out = m(input_ids=torch.from_numpy(z["input_ids"]), attention_mask=torch.from_numpy(z["attention_mask"]))
    torch.cuda.synchronize()
    assert _rel(out.last_hidden_state, z["out"]) < tol


def test_sentence_encoder_cls_pooling_and_batching():
    z = _load("mpnet_small.npz")
    enc = SentenceEncoder(model=_mpnet_from_fixture(z, "fp32"), precision="fp32")
    ids, mask = torch.from_numpy(z["input_ids"]), torch.from_numpy(z["attention_mask"])
    e = enc.encode_ids(ids, mask, batch_size=2).cpu()
    assert e.shape == (3, 64) and e.dtype == torch.float32
    assert _rel(e, torch.from_numpy(z["out"])[:, 0]) < 1e-4
    with pytest.raises(RuntimeError):
        enc.encode(["no tokenizer here"])


def test_mpnet_base_vs_oracle_l128():
    """multi-qa-mpnet-base-dot-v1 architecture (random init) at the corpus length 128 vs oracle"""
    torch.manual_seed(3)
    m = MPNetModel(MPNetConfig())
    P = {k: v.clone() for k, v in m.state_dict().items()}
    g = torch.Generator().manual_seed(4)
    ids = torch.randint(3, 30527, (2, 128), generator=g)
    mask = torch.ones_like(ids)
    mask[1, 70:] = 0
    ids[1, 70:] = 1
    ref = OE.mpnet_forward(P, ids, mask, num_layers=12, num_heads=12)
    out = m.to(DEV).set_precision("fp32")(input_ids=ids, attention_mask=mask).last_hidden_state
    assert _rel(out, ref) < 1e-3


# ---- config 5 sharded over ranks with the HIP extractors (gloo, world 2 on the box's GPU) --------
def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _corpus_files(d, n_img=11, n_txt=13):
    import numpy as np
    import pandas as pd
    from PIL import Image
    rng = np.random.default_rng(2)
    os.makedirs(os.path.join(d, "imgs"), exist_ok=True)
    for i in range(n_img):
        Image.fromarray(rng.integers(0, 256, (180 + 7 * i, 240, 3), dtype=np.uint8)).save(
            os.path.join(d, "imgs", f"im{i:02d}.jpg"), quality=92)
    from tests.toy_tokenizer import sentence
    pd.DataFrame({"id": list(range(n_txt)), "evidence_enriched": [sentence(rng, 3, 60) for _ in range(n_txt)]}).to_csv(
        os.path.join(d, "train_enriched.csv"), index=False)


def _extractors():
    from mmfd.encoders import MPNetConfig, MPNetModel
    from mmfd.evidence import ImageSimilarity, SentenceEncoder
    from tests.toy_tokenizer import toy_tokenizer
    torch.manual_seed(11)
    img = ImageSimilarity(model=resnet50(), device=DEV)  # fp32: the reference's precision
    txt = SentenceEncoder(MPNetModel(MPNetConfig()), device=DEV, tokenizer=toy_tokenizer(), max_seq_length=128)
    return img, txt


def _corpus_worker(rank, world, port, d, q):
    import torch.distributed as dist
    from tests.mp_util import watchdog
    watchdog(240)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mmfd.evidence import ImageCorpus, TextCorpus
        img, txt = _extractors()
        ImageCorpus(os.path.join(d, "sharded.pkl"), extractor=img, batch_size=4).create_feature_corpus(
            os.path.join(d, "imgs"))
        TextCorpus(d, "train", encoder=txt, out_dir=os.path.join(d, "sharded")).encode_corpus()
        q.put((rank, None))
    except BaseException:
        import traceback
        q.put((rank, traceback.format_exc()))
        raise
    finally:
        dist.destroy_process_group()


def test_sharded_corpus_build_hip_equals_single_process(tmp_path):
    """config 5 with the HIP extractors: ResNet50 + MPNet (fp32, random init) over a gloo world of 2
    ranks on the box's GPU — each rank embeds its contiguous shard of the sorted image files / CSV
    rows, rank 0 merges — gives the corpus of one process: same paths / ids in the same order,
    image features within 1e-5 and fp16 text embeddings within 1e-3 of the single-process build
    (different batch compositions are the only difference)."""
    import torch.multiprocessing as mp
    from mmfd.evidence import ImageCorpus, TextCorpus, load_corpus_pickle
    d = str(tmp_path)
    _corpus_files(d)
    os.makedirs(os.path.join(d, "single"))
    os.makedirs(os.path.join(d, "sharded"))
    img, txt = _extractors()
    single = ImageCorpus(os.path.join(d, "single.pkl"), extractor=img, batch_size=5)
    single.create_feature_corpus(os.path.join(d, "imgs"))
    one = TextCorpus(d, "train", encoder=txt, out_dir=os.path.join(d, "single")).encode_corpus()
    del img, txt
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_corpus_worker, args=(r, world, port, d, q)) for r in range(world)]
    for p in procs:
        p.start()
    from tests.mp_util import collect
    for r, err in collect(procs, q, world, deadline=260):
        assert err is None, err
    assert all(p.exitcode == 0 for p in procs)
    merged = load_corpus_pickle(os.path.join(d, "sharded.pkl"))
    assert list(merged) == list(single.feature_dict)
    for k in merged:
        a, b = merged[k], single.feature_dict[k]
        assert (a - b).abs().max().item() <= 1e-5 * b.abs().max().item(), k
    e1, i1 = TextCorpus.read(one)
    e2, i2 = TextCorpus.read(os.path.join(d, "sharded", os.path.basename(one)))
    assert i1 == i2 == [f"train_{i}" for i in range(13)]
    assert np.abs(e1.astype(np.float32) - e2.astype(np.float32)).max() <= 1e-3 * np.abs(e1.astype(np.float32)).max()
