"""Batched evidence-corpus embedding extractors on HIP kernels.

a12  ResNet50 image features — the reference's `ImageSimilarity` (im2im_retrieval.py:12-42):
     torchvision resnet50 with the classifier dropped (:14-17), eval mode, Resize(224) ->
     ToTensor -> Normalize(ImageNet) (:19-27), one image per forward (:29-36), and `ImageCorpus`
     (:45-78) looping over a directory. Here: NHWC bf16/fp32 activations, every convolution an MFMA
     GEMM (1x1 convs read the activation directly, 3x3 / strided / stem convs via an im2col
     gather), eval BatchNorm folded into the GEMM weights, ReLU and the bottleneck residual add in
     the GEMM epilogue, global average pool into fp32 features; images are processed in batches.
a13  MPNet sentence embeddings — the reference's `TextCorpus.encode_corpus` (text2text_retrieval.py:
     125-157) through SentenceTransformer("multi-qa-mpnet-base-dot-v1") = MPNetModel + CLS pooling
     (the model card's pooling; no normalisation) stored as fp16 with string ids (:144-154).

Pretrained checkpoints cannot be downloaded here: models are randomly initialised unless a
state_dict is given (torchvision / HF names load unchanged).

Corpus build (config 5): images are decoded on the host (PIL), preprocessed on the GPU in batches
(mmfd.preprocess, bit-exact with the reference's torchvision transform) and embedded in batches;
with torch.distributed initialised (or an explicit shard=(rank, world)) every rank embeds one
contiguous shard of the sorted corpus and writes its own shard file, and rank 0 merges them — no
collective on the data path. The reference's pickle corpus (path -> fp32 [2048] tensor,
im2im_retrieval.py:51-58, 78) is read with a restricted unpickler that only rebuilds tensors
(`load_corpus_pickle`) and written in the same format.
"""
from __future__ import annotations

import collections
import io
import os
import pickle

import numpy as np
import torch
import torch.nn as nn

from . import blocks as Bk
from . import kernels as K
from .encoders import MPNetConfig, MPNetModel

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


# -------------------------------------------------------------------------------------------------
# corpus files: the reference's pickle (path -> tensor) through an unpickler that executes nothing
# but tensor reconstruction, and shard bookkeeping
# -------------------------------------------------------------------------------------------------
def _storage_from_bytes(data):
    import torch as _t
    return _t.load(io.BytesIO(data), weights_only=True)


_CORPUS_ALLOWED = {
    ("torch._utils", "_rebuild_tensor_v2"): torch._utils._rebuild_tensor_v2,
    ("torch.storage", "_load_from_bytes"): _storage_from_bytes,
    ("collections", "OrderedDict"): collections.OrderedDict,
}


class _CorpusUnpickler(pickle.Unpickler):
    def find_class(self, module, name):
        fn = _CORPUS_ALLOWED.get((module, name))
        if fn is None:
            raise pickle.UnpicklingError(f"corpus pickle references {module}.{name}: only tensors are allowed")
        return fn


def load_corpus_pickle(path):
    """The reference's feature corpus (pickle.dump of {path: tensor}, im2im_retrieval.py:51-58, 78)
    -> dict; tensors are rebuilt with torch.load(weights_only=True), any other global refuses."""
    with open(path, "rb") as f:
        data = f.read()
    if not data:
        return {}
    d = _CorpusUnpickler(io.BytesIO(data)).load()
    if not isinstance(d, dict):
        raise pickle.UnpicklingError("corpus pickle does not hold a dict")
    return d


def save_corpus_pickle(path, feature_dict):
    """same format as the reference's save_features (im2im_retrieval.py:60-62)"""
    with open(path, "wb") as f:
        pickle.dump({k: torch.as_tensor(v).detach().cpu() for k, v in feature_dict.items()}, f)


def dist_shard():
    """(rank, world) of the initialised default process group, else (0, 1)"""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def shard_range(n, rank, world):
    """contiguous [lo, hi) of n items for `rank` (the first n % world ranks take one more)"""
    q, r = divmod(n, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (rank < r)


def shard_path(path, rank, world):
    root, ext = os.path.splitext(path)
    return f"{root}.shard{rank}-of-{world}{ext}"


def _barrier():
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.barrier()


# -------------------------------------------------------------------------------------------------
# ResNet50 (torchvision layout and parameter names)
# -------------------------------------------------------------------------------------------------
class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=False):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride=stride, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.stride = stride
        if downsample:
            self.downsample = nn.Sequential(nn.Conv2d(inplanes, planes * 4, 1, stride=stride, bias=False),
                                            nn.BatchNorm2d(planes * 4))
        else:
            self.downsample = None


class ResNet(nn.Module):
    """torchvision ResNet with Bottleneck blocks (resnet50: depths (3, 4, 6, 3), width 64).
    forward(x [N, 3, H, W] fp32, normalised) -> [N, 2048, 1, 1], i.e. the reference's
    nn.Sequential(*list(resnet50.children())[:-1]) (im2im_retrieval.py:15-17)."""

    def __init__(self, depths=(3, 4, 6, 3), width=64, num_classes=1000):
        super().__init__()
        self.depths, self.width = tuple(depths), width
        self.conv1 = nn.Conv2d(3, width, 7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(width)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        inplanes = width
        for i, d in enumerate(depths):
            planes = width * (2 ** i)
            stride = 1 if i == 0 else 2
            blocks = [Bottleneck(inplanes, planes, stride, downsample=(stride != 1 or inplanes != planes * 4))]
            inplanes = planes * 4
            blocks += [Bottleneck(inplanes, planes) for _ in range(1, d)]
            setattr(self, f"layer{i + 1}", nn.Sequential(*blocks))
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(inplanes, num_classes)  # unused by the extractor; kept for state_dict parity
        self.out_features = inplanes
        self.compute_dtype = torch.float32
        self._prep = None
        self._prep_key = None
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
        self.eval()

    def set_precision(self, precision):
        self.compute_dtype = {"fp32": torch.float32, "bf16": torch.bfloat16}[precision]
        self._prep = None
        return self

    def invalidate_caches(self):
        """drop the folded GEMM weights (after writes that bypass torch's version counter)"""
        self._prep = None
        return self

    def load_state_dict(self, *a, **kw):
        r = super().load_state_dict(*a, **kw)
        self._prep = None
        return r

    # ---- folded GEMM weights (recomputed when any parameter/buffer changes) --------------------
    def _prepared(self):
        tensors = list(self.parameters()) + list(self.buffers())
        key = (self.compute_dtype, tuple((t.data_ptr(), t._version) for t in tensors))
        if self._prep is not None and self._prep_key == key:
            return self._prep
        dt = self.compute_dtype

        def fold(conv, bn, kpad=None):
            w = conv.weight.detach().float().contiguous()
            return K.conv_weight_prep(w, dt, Kpad=kpad, eps=bn.eps,
                                      bn=(bn.weight.detach().float().contiguous(), bn.bias.detach().float().contiguous(),
                                          bn.running_mean.float().contiguous(), bn.running_var.float().contiguous()))

        prep = {"stem": fold(self.conv1, self.bn1, kpad=_round_up(7 * 7 * 3, 8)), "blocks": []}
        for i in range(len(self.depths)):
            for blk in getattr(self, f"layer{i + 1}"):
                prep["blocks"].append(dict(
                    c1=fold(blk.conv1, blk.bn1), c2=fold(blk.conv2, blk.bn2), c3=fold(blk.conv3, blk.bn3),
                    ds=fold(blk.downsample[0], blk.downsample[1]) if blk.downsample is not None else None,
                    stride=blk.stride, planes=blk.conv1.out_channels, cin=blk.conv1.in_channels))
        self._prep, self._prep_key = prep, key
        return prep

    @torch.no_grad()
    def forward(self, x):
        dev = self.conv1.weight.device
        if dev.type != "cuda":
            raise RuntimeError("mmfd ResNet runs on the HIP device: call .to('cuda') first")
        x = x.to(dev, torch.float32).contiguous()
        N = x.shape[0]
        prep = self._prepared()
        dt = self.compute_dtype
        w, b = prep["stem"]
        cols, H, W = K.im2col_nchw(x, 7, 2, 3, w.shape[1], dt)
        y = K.gemm(cols, w, bias=b, act=K.ACT_RELU)
        del cols
        y, H, W = K.maxpool_nhwc(y, N, H, W, self.width)
        for blk in prep["blocks"]:
            y, H, W = _bottleneck(y, N, H, W, blk)
        feats = K.global_avgpool(y, N, H * W, y.shape[1])
        return feats.view(N, -1, 1, 1)


def _round_up(x, m):
    return (x + m - 1) // m * m


# the 3x3 and strided 1x1 convolutions as implicit GEMMs (the GEMM's operand fill gathers the
# windows; no im2col matrix); MMFD_CONV_IM2COL=1 restores the explicit im2col + GEMM (A/B runs)
IMPLICIT_CONV = os.environ.get("MMFD_CONV_IM2COL") != "1"


def _conv(x, N, H, W, C, w, b, k, s, pad, act=K.ACT_NONE):
    """conv(k x k, stride s, pad) of NHWC rows x [N*H*W, C] with the folded weight w [Cout, k*k*C]:
    implicit GEMM where the channel count allows it, else im2col + GEMM. Returns (y, Ho, Wo)."""
    if IMPLICIT_CONV and K.conv_implicit_ok(x.dtype, C) and w.shape[1] == k * k * C:
        return K.conv2d_nhwc(x, N, H, W, C, w, k, s, pad, bias=b, act=act)
    cols, Ho, Wo = K.im2col_nhwc(x, N, H, W, C, k, s, pad, Kpad=w.shape[1])
    return K.gemm(cols, w, bias=b, act=act), Ho, Wo


def _bottleneck(x, N, H, W, blk):
    """relu(bn3(conv3(relu(bn2(conv2(relu(bn1(conv1 x))))))) + shortcut(x)) on NHWC rows"""
    s, planes, cin = blk["stride"], blk["planes"], blk["cin"]
    w1, b1 = blk["c1"]
    h1 = K.gemm(x, w1, bias=b1, act=K.ACT_RELU)                          # 1x1
    w2, b2 = blk["c2"]
    h2, Ho, Wo = _conv(h1, N, H, W, planes, w2, b2, 3, s, 1, act=K.ACT_RELU)  # 3x3 (stride s)
    del h1
    if blk["ds"] is not None:
        wd, bd = blk["ds"]
        if s == 1:
            ident = K.gemm(x, wd, bias=bd)                                # 1x1 + BN
        else:
            ident = _conv(x, N, H, W, cin, wd, bd, 1, s, 0)[0]            # 1x1 stride s + BN
    else:
        ident = x
    w3, b3 = blk["c3"]
    y = K.gemm(h2, w3, bias=b3, act=K.ACT_RELU, residual=ident, residual_first=True)
    return y, Ho, Wo


def resnet50(**kw):
    return ResNet((3, 4, 6, 3), 64, **kw)


# -------------------------------------------------------------------------------------------------
# image preprocessing (im2im_retrieval.py:19-27) and the extractor API
# -------------------------------------------------------------------------------------------------
def _decode(image):
    """host decode (PIL) -> RGB PIL image (the file is read and closed here)"""
    from PIL import Image
    if not isinstance(image, Image.Image):
        with Image.open(image) as im:
            return im.convert("RGB")
    return image.convert("RGB")


class ImageSimilarity:
    """im2im_retrieval.py:12-42 — ResNet50 features of one image (`extract_features`) plus the
    batched `extract_batch` the corpus build uses."""

    def __init__(self, state_dict=None, device="cuda", precision="fp32", model=None):
        # fp32 by default: the reference extracts in fp32 (im2im_retrieval.py:14-36); "bf16" is the
        # faster option
        self.model = model if model is not None else resnet50()
        if state_dict is not None:  # a torchvision resnet50 checkpoint: its fc layer is dropped (:14-17)
            Bk.load_state_dict_checked(self.model, state_dict, benign=("fc", "num_batches_tracked"))
        self.model = self.model.to(device).eval().set_precision(precision)
        self.device = device
        self._pre = None

    def preprocess_batch(self, images):
        """decoded images (PIL / uint8 HWC) -> normalised fp32 [N, 3, 224, 224] on the device: the
        transform of im2im_retrieval.py:19-27 on the GPU (mmfd.preprocess "retrieval", bit-exact)"""
        if self._pre is None:
            from .preprocess import ImagePreprocessor
            self._pre = ImagePreprocessor("retrieval", device=self.device)
        return self._pre(images)

    def preprocess_device(self, src, shapes, offsets):
        """decoded uint8 HWC pixels already in the device buffer `src` -> normalised fp32 [N, 3, 224,
        224] (the "retrieval" transform; see ImagePreprocessor.from_device)"""
        if self._pre is None:
            from .preprocess import ImagePreprocessor
            self._pre = ImagePreprocessor("retrieval", device=self.device)
        return self._pre.from_device(src, shapes, offsets)

    def extract_batch(self, pixels):
        """normalised fp32 [N, 3, 224, 224] (host or device) -> fp32 [N, 2048] on the device"""
        return self.model(pixels).flatten(1)

    def extract_features(self, image_stream):
        """im2im_retrieval.py:29-36: one image (path / stream) -> fp32 [2048] (host)"""
        x = self.preprocess_batch([_decode(image_stream)])
        return self.extract_batch(x).flatten().cpu()

    @staticmethod
    def similarity(features1, features2):
        f1, f2 = features1.double().flatten(), features2.double().flatten()
        den = max(float(f1.norm() * f2.norm()), 1e-6)  # nn.CosineSimilarity(dim=1, eps=1e-6)
        return float((f1 @ f2) / den)


class ImageCorpus:
    """im2im_retrieval.py:45-78 with batched GPU extraction. The corpus file is the reference's
    pickle (path -> fp32 [2048] tensor) unless its name ends in .npz (`paths`, `features`)."""

    def __init__(self, feature_corpus_path, extractor: ImageSimilarity | None = None, batch_size=256,
                 decode_workers=None, decode="processes"):
        self.feature_corpus_path = feature_corpus_path
        self.feature_extractor = extractor or ImageSimilarity()
        self.batch_size = batch_size
        # host decode workers: the next batch is decoded while the GPU preprocesses and embeds the
        # current one. "processes" (default): a forkserver process pool handing the pixels back in
        # shared memory (mmfd.hostdecode; PIL holds the GIL outside its decoder, which capped the
        # thread pool at ~1.6k images/s); "threads": the thread pool of round 3
        self.decode_workers = decode_workers or min(16, len(os.sched_getaffinity(0)))
        if decode not in ("processes", "threads"):
            raise ValueError("decode must be 'processes' or 'threads'")
        self.decode = decode
        self._pool = None
        self.feature_dict = self.load_features()
        self._revision = 0  # bumped on every feature_dict write: the device index is rebuilt

    @staticmethod
    def _read(path):
        if not os.path.exists(path):
            return {}
        if path.endswith(".npz"):
            z = np.load(path, allow_pickle=False)
            return {p: torch.from_numpy(f) for p, f in zip(z["paths"].tolist(), z["features"])}
        return load_corpus_pickle(path)

    @staticmethod
    def _write(path, feature_dict):
        if path.endswith(".npz"):
            paths = list(feature_dict)
            feats = (np.stack([torch.as_tensor(feature_dict[p]).numpy() for p in paths]) if paths
                     else np.zeros((0, 2048), np.float32))
            with open(path, "wb") as f:
                np.savez(f, paths=np.array(paths), features=feats)
        else:
            save_corpus_pickle(path, feature_dict)

    def load_features(self):
        return self._read(self.feature_corpus_path)

    def save_features(self):
        self._write(self.feature_corpus_path, self.feature_dict)

    def add_image(self, image_path):
        self.feature_dict[image_path] = self.feature_extractor.extract_features(image_path)
        self._revision += 1
        self.save_features()

    def _decode_pool(self):
        if self._pool is None:
            from .hostdecode import DecodePool
            self._pool = DecodePool(self.decode_workers)
        return self._pool

    def close(self):
        """stop the decode worker processes (they are otherwise kept for the next build)"""
        if self._pool is not None:
            self._pool.close()
            self._pool = None
        if getattr(self, "_ring", None) is not None:
            self._ring.close()
            self._ring = None

    def _decode_ring(self):
        ring = getattr(self, "_ring", None)
        if ring is None or ring.gps * ring.group < self.batch_size:
            from .hostdecode import PinnedDecodeRing
            if ring is not None:
                ring.close()
            ring = self._ring = PinnedDecodeRing(self.batch_size, self.feature_extractor.device, self.decode_workers)
        return ring

    def _extract_paths(self, paths):
        out = {}
        chunks = [paths[i:i + self.batch_size] for i in range(0, len(paths), self.batch_size)]
        if not chunks:
            return out
        ex = self.feature_extractor
        ring = None
        if (self.decode == "processes" and self.decode_workers > 1 and hasattr(ex, "preprocess_device")
                and torch.device(ex.device).type == "cuda"):
            from .hostdecode import RingUnavailable
            try:
                ring = self._decode_ring()
            except RingUnavailable as err:  # no shared memory / page locking here: the process pool
                import warnings
                warnings.warn(f"{err}; decoding through the process pool instead")
                self.decode_ring_error = str(err)
        if ring is not None:
            # the workers decode into a page-locked shared ring, the batch's pixels go to the device
            # with asynchronous copies, and the features stay on the device until the build is done:
            # the host thread only submits and enqueues, so decode, upload and the GPU overlap
            h = ring.submit(chunks[0], 0)
            feats = []
            for ci, chunk in enumerate(chunks):
                src, shapes, offs = ring.upload(h, ci % 2)
                if ci + 1 < len(chunks):
                    h = ring.submit(chunks[ci + 1], (ci + 1) % 2)
                feats.append(ex.extract_batch(ex.preprocess_device(src, shapes, offs)).float())
            allf = torch.cat(feats).cpu()
            return {p: allf[i].clone() for i, p in enumerate(paths)}
        if self.decode == "processes" and self.decode_workers > 1:
            pool = self._decode_pool()
            nxt = pool.submit(chunks[0])
            for ci, chunk in enumerate(chunks):
                imgs, release = pool.get(nxt)
                if ci + 1 < len(chunks):  # decode the next batch on the host while this one runs
                    nxt = pool.submit(chunks[ci + 1])
                px = self.feature_extractor.preprocess_batch(imgs)  # copies the pixels (pinned upload)
                del imgs
                release()
                feats = self.feature_extractor.extract_batch(px).float().cpu()
                for p, f in zip(chunk, feats):
                    out[p] = f.clone()
            return out
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(max_workers=max(1, self.decode_workers)) as pool:
            nxt = [pool.submit(_decode, p) for p in chunks[0]]
            for ci, chunk in enumerate(chunks):
                imgs = [f.result() for f in nxt]
                if ci + 1 < len(chunks):  # decode the next batch on the host while this one runs
                    nxt = [pool.submit(_decode, p) for p in chunks[ci + 1]]
                px = self.feature_extractor.preprocess_batch(imgs)
                feats = self.feature_extractor.extract_batch(px).float().cpu()
                for p, f in zip(chunk, feats):
                    out[p] = f.clone()
        return out

    def create_feature_corpus(self, image_dir, shard=None):
        """im2im_retrieval.py:69-78 over the .png/.jpg/.jpeg files of image_dir, in batches. With a
        process group (or shard=(rank, world)) each rank embeds its contiguous shard of the sorted
        file list into `<corpus>.shard<r>-of-<w>` and rank 0 merges the shards into the corpus."""
        paths = [os.path.join(image_dir, n) for n in sorted(os.listdir(image_dir))]
        paths = [p for p in paths if os.path.isfile(p) and p.lower().endswith((".png", ".jpg", ".jpeg"))]
        rank, world = shard if shard is not None else dist_shard()
        if world == 1:
            self.feature_dict.update(self._extract_paths(paths))
            self._revision += 1
            self.save_features()
            return self.feature_corpus_path
        lo, hi = shard_range(len(paths), rank, world)
        self._write(shard_path(self.feature_corpus_path, rank, world), self._extract_paths(paths[lo:hi]))
        if shard is None:
            _barrier()
            if rank == 0:
                self.merge_shards(world)
            _barrier()
            self.feature_dict = self.load_features()
            self._revision += 1
        return shard_path(self.feature_corpus_path, rank, world)

    def merge_shards(self, world, remove=True):
        """rank 0: concatenate the per-rank shard files (in rank order) into the corpus file"""
        for r in range(world):
            sp = shard_path(self.feature_corpus_path, r, world)
            self.feature_dict.update(self._read(sp))
            if remove:
                os.remove(sp)
        self._revision += 1
        self.save_features()

    def index(self):
        """The corpus features as a device-resident CorpusIndex (rebuilt when the corpus changed)."""
        from .retrieval import CorpusIndex
        key = (id(self.feature_dict), self._revision, len(self.feature_dict))
        if getattr(self, "_index_key", None) != key:
            paths = list(self.feature_dict)
            feats = torch.stack([self.feature_dict[p].float().flatten() for p in paths])
            self._index = CorpusIndex(feats, ids=paths, device=self.feature_extractor.device, mode="pair", eps=1e-6)
            self._index_key = key
        return self._index

    def retrieve_similar_images(self, query_image_path, top_k=50):
        """im2im_retrieval.py:80-106: [(path, score)] of the top_k corpus images with distinct
        cosine scores, best first (scores and ranking on the GPU: retrieval.CorpusIndex)."""
        q = self.feature_extractor.extract_features(query_image_path)
        return self.index().search(q.float().unsqueeze(0).to(self.feature_extractor.device), top_k)[0]


# -------------------------------------------------------------------------------------------------
# text corpus (text2text_retrieval.py:123-157)
# -------------------------------------------------------------------------------------------------
class SentenceEncoder:
    """MPNet + CLS pooling (SentenceTransformer("multi-qa-mpnet-base-dot-v1").encode semantics on
    token ids). `encode(texts)` needs a tokenizer object (none can be downloaded here)."""

    def __init__(self, model: MPNetModel | None = None, state_dict=None, device="cuda", precision="fp32",
                 tokenizer=None, max_seq_length=512):
        self.model = model if model is not None else MPNetModel(MPNetConfig())
        if state_dict is not None:  # sentence-transformers' MPNet checkpoints carry an unused pooler
            Bk.load_state_dict_checked(self.model, state_dict, benign=("pooler", "position_ids"))
        self.model = self.model.to(device).eval().set_precision(precision)
        self.tokenizer = tokenizer
        self.max_seq_length = max_seq_length

    def encode_ids(self, input_ids, attention_mask=None, batch_size=256):
        """int64 [N, L] -> fp32 [N, 768] CLS embeddings (device)"""
        outs = []
        for i in range(0, input_ids.shape[0], batch_size):
            ids = input_ids[i:i + batch_size]
            m = attention_mask[i:i + batch_size] if attention_mask is not None else None
            h = self.model(input_ids=ids, attention_mask=m).last_hidden_state
            outs.append(K.cast(h[:, 0].contiguous(), torch.float32))
        return torch.cat(outs) if len(outs) > 1 else outs[0]

    def encode(self, sentences, batch_size=256, convert_to_tensor=True):
        """SentenceTransformer.encode: a str gives [768], a list [N, 768] (fp32, host). As
        sentence-transformers does, the texts are tokenised once, sorted by length and encoded in
        batches padded to their own longest text (CLS pooling over masked keys: the padding
        length does not change an embedding), then returned in input order."""
        if self.tokenizer is None:
            raise RuntimeError("SentenceEncoder.encode needs a tokenizer (pass tokenizer=...); use encode_ids")
        single = isinstance(sentences, str)
        texts = [sentences] if single else list(sentences)
        if not texts:
            emb = torch.zeros(0, self.model.config.hidden_size)
            return emb if convert_to_tensor else emb.numpy()
        ids = self.tokenizer(texts, truncation=True, max_length=self.max_seq_length)["input_ids"]
        order = sorted(range(len(ids)), key=lambda i: -len(ids[i]))
        pad = getattr(self.tokenizer, "pad_token_id", 0) or 0
        out = torch.empty(len(ids), self.model.config.hidden_size)
        for i in range(0, len(order), batch_size):
            idx = order[i:i + batch_size]
            L = len(ids[idx[0]])
            x = torch.full((len(idx), L), pad, dtype=torch.int64)
            m = torch.zeros((len(idx), L), dtype=torch.int64)
            for r, j in enumerate(idx):
                x[r, :len(ids[j])] = torch.tensor(ids[j])
                m[r, :len(ids[j])] = 1
            dev = self.model_device()
            out[idx] = self.encode_ids(x.to(dev, non_blocking=True), m.to(dev, non_blocking=True), batch_size).cpu()
        emb = out[0] if single else out
        return emb if convert_to_tensor else emb.numpy()

    def model_device(self):
        return next(self.model.parameters()).device


class TextCorpus:
    """text2text_retrieval.py:123-157: encode `{split}_enriched.csv`'s evidence_enriched column and
    store fp16 embeddings with ids `{split}_{id}` (HDF5 when h5py is importable, else .npz)."""

    def __init__(self, data_dir, split, encoder: SentenceEncoder | None = None, out_dir=None):
        self.bi_encoder = encoder or SentenceEncoder()
        self.split, self.data_dir = split, data_dir
        self.out_dir = out_dir or data_dir

    def encode_corpus(self, shard=None):
        """text2text_retrieval.py:129-157. With a process group (or shard=(rank, world)) each rank
        encodes its contiguous shard of the CSV rows into a shard file and rank 0 concatenates the
        shards (rank order = row order) into `{split}_embeddings.{h5|npz}`."""
        import pandas as pd
        df = pd.read_csv(os.path.join(self.data_dir, f"{self.split}_enriched.csv"))
        texts = df["evidence_enriched"].tolist()
        ids = [f"{self.split}_{i}" for i in df["id"].tolist()]
        rank, world = shard if shard is not None else dist_shard()
        lo, hi = shard_range(len(texts), rank, world)
        emb = self.bi_encoder.encode(texts[lo:hi]).numpy().astype(np.float16) if hi > lo else \
            np.zeros((0, 768), np.float16)
        path = self.output_path()
        if world == 1:
            return self._write(path, emb, ids)
        self._write(shard_path(path, rank, world), emb, ids[lo:hi])
        if shard is None:
            _barrier()
            if rank == 0:
                self.merge_shards(world)
            _barrier()
        return path if shard is None else shard_path(path, rank, world)

    def output_path(self):
        try:
            import h5py  # noqa: F401
            ext = "h5"
        except ImportError:
            ext = "npz"
        return os.path.join(self.out_dir, f"{self.split}_embeddings.{ext}")

    @staticmethod
    def _write(path, emb, ids):
        if path.endswith(".h5"):
            import h5py
            with h5py.File(path, "w") as h5:
                h5.create_dataset("embeddings", data=emb, dtype="float16")
                h5.create_dataset("ids", data=ids, dtype=h5py.string_dtype())
        else:
            with open(path, "wb") as f:
                np.savez(f, embeddings=emb, ids=np.array(ids, dtype=str))
        return path

    @staticmethod
    def read(path):
        """(fp16 embeddings [N, 768], ids) of an embeddings file (text2text_retrieval.py:39-47)"""
        if path.endswith(".h5"):
            import h5py
            with h5py.File(path, "r") as h5:
                return h5["embeddings"][()], [x.decode() if isinstance(x, bytes) else x for x in h5["ids"][()]]
        z = np.load(path, allow_pickle=False)
        return z["embeddings"], z["ids"].tolist()

    def merge_shards(self, world, remove=True):
        path = self.output_path()
        embs, ids = [], []
        for r in range(world):
            sp = shard_path(path, r, world)
            e, i = self.read(sp)
            embs.append(e)
            ids += list(i)
            if remove:
                os.remove(sp)
        return self._write(path, np.concatenate(embs) if embs else np.zeros((0, 768), np.float16), ids)
