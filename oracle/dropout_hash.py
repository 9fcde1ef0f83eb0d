"""TEST INFRASTRUCTURE ONLY (oracle). Never imported by the product path.

numpy restatement of the counter-based dropout hash used by every mmfd kernel
(multimodal-misinformation-detection_amd/csrc/common.h: mmfd_mix32 / mmfd_hash /
mmfd_drop_threshold). The reference draws dropout masks from torch's RNG (layers.py:15,17,53;
model.py:255-288); torch's CPU and GPU streams differ anyway, so parity in train mode is checked
against THIS mask: the oracle applies the same mask to the reference math.
"""
import numpy as np

_M1 = np.uint32(0x7FEB352D)
_M2 = np.uint32(0x846CA68B)


def mix32(x):
    x = np.asarray(x, dtype=np.uint32)
    with np.errstate(over="ignore"):
        x = x ^ (x >> np.uint32(16))
        x = (x * _M1).astype(np.uint32)
        x = x ^ (x >> np.uint32(15))
        x = (x * _M2).astype(np.uint32)
        x = x ^ (x >> np.uint32(16))
    return x


def _key(seed: int, salt: int):
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    salt = int(salt) & 0xFFFFFFFFFFFFFFFF
    k0 = mix32(np.uint32(seed & 0xFFFFFFFF) ^ mix32(np.uint32(seed >> 32) ^ np.uint32(0x85EBCA6B)))
    return mix32(k0 ^ np.uint32(salt & 0xFFFFFFFF) ^ mix32(np.uint32(salt >> 32) ^ np.uint32(0xC2B2AE35)))


def dropout_hash(seed: int, salt: int, idx):
    """mmfd_hash(seed, salt, idx) = mix32(key ^ lo*0x9E3779B1 ^ hi*0x85EBCA77), key = mmfd_hash_key"""
    idx = np.asarray(idx, dtype=np.uint64)
    lo = (idx & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    hi = (idx >> np.uint64(32)).astype(np.uint32)
    with np.errstate(over="ignore"):
        x = (lo * np.uint32(0x9E3779B1)).astype(np.uint32) ^ (hi * np.uint32(0x85EBCA77)).astype(np.uint32)
        return mix32(_key(seed, salt) ^ x)


def drop_threshold(p: float) -> int:
    t = float(np.float32(p)) * 4294967296.0
    if t >= 4294967295.0:
        return 0xFFFFFFFF
    return int(t)


def keep_mask(seed: int, salt: int, shape, p: float):
    """Boolean keep-mask for a contiguous tensor of `shape` (element index = flat index)."""
    n = int(np.prod(shape))
    h = dropout_hash(seed, salt, np.arange(n, dtype=np.uint64))
    return (h >= np.uint32(drop_threshold(p))).reshape(shape)


def salt_of(name: str) -> int:
    """Call-site id (same formula as the product's kernels.salt_of; checked by the tests)."""
    import zlib

    b = name.encode()
    return (zlib.crc32(b) << 32) | zlib.crc32(b[::-1] + b"mmfd")


def drop_threshold16(p: float) -> int:
    """attention kernels' 16-bit threshold (common.h mmfd_drop_threshold16): round(p * 65536)"""
    t = float(np.float32(p)) * 65536.0 + 0.5
    return 65536 if t >= 65536.0 else int(t)


def attn_keep_mask(seed: int, salt: int, shape, p: float, rows=None):
    """Keep-mask of attention probabilities [B, H, Lq, Lk] as the attention kernels draw it
    (multimodal-misinformation-detection_amd/csrc/attention.hip pair_keep): ONE hash per key pair,
    h = hash(row * kp + k // 2) with row = (b*H + h)*Lq + q and kp = ceil(Lk / 2); element (row, k) is
    kept when its 16-bit half (low for even k, high for odd k) >= round(p * 65536). `rows`: the
    whole-batch indices of the tensor's batch rows (chunked oracle steps; default arange(B))."""
    B, H, Lq, Lk = (int(x) for x in shape)
    rows = np.arange(B, dtype=np.uint64) if rows is None else np.asarray(rows, dtype=np.uint64)
    kp = np.uint64((Lk + 1) // 2)
    r = ((rows[:, None, None] * np.uint64(H) + np.arange(H, dtype=np.uint64)[None, :, None]) * np.uint64(Lq)
         + np.arange(Lq, dtype=np.uint64)[None, None, :])
    k = np.arange(Lk, dtype=np.uint64)
    pidx = r[..., None] * kp + (k >> np.uint64(1))[None, None, None, :]
    h = dropout_hash(seed, salt, pidx.reshape(-1)).reshape(B, H, Lq, Lk).astype(np.int64)
    half = np.where((k & np.uint64(1)).astype(bool)[None, None, None, :], h >> 16, h & 0xFFFF)
    return half >= drop_threshold16(p)


def keep_mask_rows(seed: int, salt: int, shape, p: float, rows):
    """Keep-mask of a batch-major contiguous tensor of `shape` that holds the batch rows `rows` of a
    larger whole batch: element e of batch row r has the whole-batch flat index
    rows[r] * inner + e (inner = numel / len(rows)) — the index the HIP kernels hash when they run
    the whole batch at once. rows = arange(R) is keep_mask."""
    rows = np.asarray(rows, dtype=np.uint64)
    n = int(np.prod(shape))
    assert n % len(rows) == 0, (shape, len(rows))
    inner = n // len(rows)
    idx = rows[:, None] * np.uint64(inner) + np.arange(inner, dtype=np.uint64)[None, :]
    h = dropout_hash(seed, salt, idx.reshape(-1))
    return (h >= np.uint32(drop_threshold(p))).reshape(shape)


class Drop:
    """`drop(site, x)` callback for the oracle: applies exactly the HIP kernels' mask (sites ending in
    ".attn" — attention probabilities — with attn_keep_mask, every other site with keep_mask). With `rows`
    (the whole-batch row indices of this call's batch rows, see keep_mask_rows) a chunk of a larger
    batch gets the masks the whole batch gets at those rows: oracle.train_step.chunked_loss_grads
    binds one per chunk for the encoders (stacked claim|evidence rows [s:e] and [B+s:B+e]) and one
    for the head (rows [s:e])."""

    def __init__(self, seed: int, p: float, rows=None):
        self.seed, self.p, self.rows = int(seed), float(p), rows

    def with_rows(self, rows):
        return Drop(self.seed, self.p, rows)

    def __call__(self, site, x):
        import torch
        if site.endswith(".attn"):  # attention probabilities [B, H, Lq, Lk]: the pair-hash mask
            keep = attn_keep_mask(self.seed, salt_of(site), tuple(x.shape), self.p, self.rows)
        elif self.rows is None:
            keep = keep_mask(self.seed, salt_of(site), tuple(x.shape), self.p)
        else:
            keep = keep_mask_rows(self.seed, salt_of(site), tuple(x.shape), self.p, self.rows)
        return x * torch.from_numpy(keep).to(x.dtype) / (1.0 - self.p)


def make_drop(seed: int, p: float, dtype=None):
    """`drop(site, x)` callback for the oracle: applies exactly the HIP kernels' mask."""
    return Drop(seed, p)
