"""Evidence-corpus files and rank sharding on the CPU (no GPU calls).

* the reference's pickle corpus (pickle.dump of {path: tensor}, im2im_retrieval.py:51-62, 78)
  round-trips through mmfd's restricted unpickler, which refuses any other global;
* create_feature_corpus sharded over a gloo world of 2 (contiguous shards of the sorted file list,
  one shard file per rank, rank-0 merge) gives the same corpus as one process. The extractor is a
  CPU stand-in here (the oracle's preprocessing + a fixed reduction): the code under test is the
  sharding / file protocol, the HIP extractor itself is covered by tests/test_evidence_gpu.py.
"""
import os
import pickle
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


class _StubExtractor:
    device = "cpu"

    def preprocess_batch(self, images):
        from oracle.preprocess import preprocess
        from mmfd.preprocess import MODES
        c = MODES["retrieval"]
        from PIL import Image
        ims = [Image.fromarray(im) if isinstance(im, np.ndarray) else im for im in images]
        return torch.stack([torch.from_numpy(preprocess(im, c["resize"], None, c["mean"], c["std"])) for im in ims])

    def extract_batch(self, px):
        return torch.cat([px.mean(dim=(2, 3)), px.amax(dim=(2, 3))], dim=1)

    def extract_features(self, path):
        from PIL import Image
        return self.extract_batch(self.preprocess_batch([Image.open(path).convert("RGB")]))[0]


def _images(d, n=7):
    from PIL import Image
    rng = np.random.default_rng(1)
    for i in range(n):
        Image.fromarray(rng.integers(0, 255, (30 + i, 41, 3), dtype=np.uint8)).save(os.path.join(d, f"im{i:02d}.jpg"))


def test_reference_pickle_corpus_roundtrip_and_refusal(tmp_path):
    from mmfd.evidence import ImageCorpus, load_corpus_pickle
    feats = {f"/data/{i}.jpg": torch.randn(2048) for i in range(4)}
    p = tmp_path / "corpus.pkl"
    with open(p, "wb") as f:
        pickle.dump(feats, f)  # exactly what the reference's save_features writes
    got = load_corpus_pickle(str(p))
    assert list(got) == list(feats) and all(torch.equal(got[k], feats[k]) for k in feats)
    c = ImageCorpus(str(p), extractor=_StubExtractor())
    assert set(c.feature_dict) == set(feats)

    class Evil:
        def __reduce__(self):
            return (os.system, ("echo pwned",))

    bad = tmp_path / "bad.pkl"
    with open(bad, "wb") as f:
        pickle.dump({"x": Evil()}, f)
    with pytest.raises(pickle.UnpicklingError):
        load_corpus_pickle(str(bad))
    (tmp_path / "empty.pkl").write_bytes(b"")
    assert load_corpus_pickle(str(tmp_path / "empty.pkl")) == {}


def test_shard_range_covers_everything_once():
    from mmfd.evidence import shard_range
    for n in (0, 1, 7, 64, 100003):
        for w in (1, 2, 3, 8):
            spans = [shard_range(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _shard_worker(rank, world, port, d):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mmfd.evidence import ImageCorpus
        c = ImageCorpus(os.path.join(d, "sharded.pkl"), extractor=_StubExtractor(), batch_size=2)
        c.create_feature_corpus(os.path.join(d, "imgs"))
    finally:
        dist.destroy_process_group()


def test_sharded_corpus_build_equals_single_process(tmp_path):
    from mmfd.evidence import ImageCorpus, load_corpus_pickle
    os.makedirs(tmp_path / "imgs")
    _images(str(tmp_path / "imgs"))
    single = ImageCorpus(str(tmp_path / "single.pkl"), extractor=_StubExtractor(), batch_size=3)
    single.create_feature_corpus(str(tmp_path / "imgs"))
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_shard_worker, args=(r, world, port, str(tmp_path))) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    merged = load_corpus_pickle(str(tmp_path / "sharded.pkl"))
    assert list(merged) == list(single.feature_dict)  # sorted order, every file once
    for k in merged:
        assert torch.allclose(merged[k], single.feature_dict[k], atol=1e-6)
    assert not [f for f in os.listdir(tmp_path) if ".shard" in f]  # shard files merged and removed


class _StubTextEncoder:
    def encode(self, texts):
        return torch.tensor([[float(len(t)), float(sum(map(ord, t)) % 997)] + [0.0] * 766 for t in texts])


def _text_worker(rank, world, port, d):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mmfd.evidence import TextCorpus
        TextCorpus(d, "train", encoder=_StubTextEncoder(), out_dir=os.path.join(d, "sharded")).encode_corpus()
    finally:
        dist.destroy_process_group()


def test_sharded_text_corpus_equals_single_process(tmp_path):
    import pandas as pd
    from mmfd.evidence import TextCorpus
    pd.DataFrame({"id": list(range(11)), "evidence_enriched": [f"evidence text {i} " * (i + 1) for i in range(11)]}
                 ).to_csv(tmp_path / "train_enriched.csv", index=False)
    os.makedirs(tmp_path / "single")
    os.makedirs(tmp_path / "sharded")
    one = TextCorpus(str(tmp_path), "train", encoder=_StubTextEncoder(), out_dir=str(tmp_path / "single")).encode_corpus()
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_text_worker, args=(r, world, port, str(tmp_path))) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    e1, i1 = TextCorpus.read(one)
    e2, i2 = TextCorpus.read(str(tmp_path / "sharded" / os.path.basename(one)))
    assert i1 == i2 == [f"train_{i}" for i in range(11)]
    assert e1.dtype == np.float16 and np.array_equal(e1, e2)


def test_process_pool_decode_is_bit_exact(tmp_path, monkeypatch):
    """mmfd.hostdecode.DecodePool (worker processes, pixels returned in shared memory) returns exactly
    the bytes of evidence._decode (PIL open + convert("RGB")) for JPEG / PNG / grayscale / RGBA /
    palette files, in submission order, and leaves none of its shared-memory blocks behind (the
    blocks this pool handed back are tracked by name, so tests running beside it under xdist do not
    count)."""
    from multiprocessing import shared_memory

    from PIL import Image

    import mmfd.hostdecode as hd
    from mmfd.evidence import _decode
    from mmfd.hostdecode import DecodePool
    seen = []

    class _Tracked(shared_memory.SharedMemory):
        def __init__(self, name=None, create=False, size=0):
            super().__init__(name=name, create=create, size=size)
            seen.append(self.name.lstrip("/"))

    monkeypatch.setattr(hd.shared_memory, "SharedMemory", _Tracked)
    rng = np.random.default_rng(7)
    paths = []
    for i, (mode, ext) in enumerate([("RGB", "jpg"), ("RGB", "png"), ("L", "jpg"), ("RGBA", "png"), ("P", "png"),
                                     ("RGB", "jpeg"), ("L", "png")] * 3):
        h, w = 17 + 5 * i, 23 + 3 * i
        a = rng.integers(0, 255, (h, w, 4 if mode == "RGBA" else 3), dtype=np.uint8)
        im = Image.fromarray(a, "RGBA" if mode == "RGBA" else "RGB")
        if mode in ("L", "P"):
            im = im.convert(mode)
        p = str(tmp_path / f"x{i:02d}.{ext}")
        im.save(p)
        paths.append(p)
    pool = DecodePool(workers=3, group=4)
    try:
        h1 = pool.submit(paths[:10])
        h2 = pool.submit(paths[10:])
        for h, ps in ((h1, paths[:10]), (h2, paths[10:])):
            views, release = pool.get(h)
            assert len(views) == len(ps)
            for v, p in zip(views, ps):
                want = np.asarray(_decode(p))
                assert v.dtype == np.uint8 and v.shape == want.shape and np.array_equal(v, want), p
            del v, views
            release()
        with pytest.raises(Exception):
            pool.get(pool.submit([str(tmp_path / "missing.jpg")]))
    finally:
        pool.close()
    assert len(seen) == 6  # one block per 4-path group: 3 for the first 10 paths, 3 for the last 11
    if os.path.isdir("/dev/shm"):
        assert set(seen) & set(os.listdir("/dev/shm")) == set()


def test_corpus_decode_processes_equals_threads(tmp_path):
    from mmfd.evidence import ImageCorpus
    os.makedirs(tmp_path / "imgs")
    _images(str(tmp_path / "imgs"), n=9)
    a = ImageCorpus(str(tmp_path / "p.pkl"), extractor=_StubExtractor(), batch_size=4, decode_workers=3)
    b = ImageCorpus(str(tmp_path / "t.pkl"), extractor=_StubExtractor(), batch_size=4, decode_workers=3,
                    decode="threads")
    try:
        a.create_feature_corpus(str(tmp_path / "imgs"))
        b.create_feature_corpus(str(tmp_path / "imgs"))
    finally:
        a.close()
    assert list(a.feature_dict) == list(b.feature_dict)
    assert all(torch.equal(a.feature_dict[k], b.feature_dict[k]) for k in a.feature_dict)
