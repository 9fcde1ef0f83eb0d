"""Data parallelism (BASELINE config 4): one process per GPU, gradients averaged with RCCL over xGMI.

The reference is single-device (train.py:321); the batch dimension shards naturally (independent
claim/evidence pairs), so each rank runs the full step on its own 256 pairs and the only exchange is
the gradient all-reduce. Gradients are packed into ~64 MB fp32 buckets (few, large collectives suit
the point-to-point xGMI rings), all-reduced with op AVG, and unpacked.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import kernels as K


def _pack(g, dst):
    K.cast(g, torch.float32, out=dst)


def _unpack(src, g, scale):
    K.axpby(scale, src, 0.0, None, out=g)


class GradAllReduce:
    """`pack(grad, flat_slice)` / `unpack(flat_slice, grad, scale)` default to the HIP cast/axpby
    kernels; they are parameters only so the bucketing + collective logic can be exercised on the
    CPU (gloo) in tests."""

    def __init__(self, bucket_mb: float = 64.0, group=None, pack=_pack, unpack=_unpack):
        self.bucket_elems = max(1, int(bucket_mb * (1 << 20) / 4))
        self.group = group
        self._bufs = {}
        self._pack, self._unpack = pack, unpack

    def _buckets(self, grads):
        bucket, n = [], 0
        for g in grads:
            if bucket and n + g.numel() > self.bucket_elems:
                yield bucket, n
                bucket, n = [], 0
            bucket.append(g)
            n += g.numel()
        if bucket:
            yield bucket, n

    def allreduce_grads(self, params):
        grads = [p.grad for p in params if p.grad is not None]
        if not grads or not dist.is_initialized() or dist.get_world_size(self.group) == 1:
            return
        world = dist.get_world_size(self.group)
        works = []
        for i, (bucket, n) in enumerate(self._buckets(grads)):
            buf = self._bufs.get(i)
            if buf is None or buf.numel() < n or buf.device != bucket[0].device:
                buf = self._bufs[i] = torch.empty(n, device=bucket[0].device, dtype=torch.float32)
            off = 0
            for g in bucket:
                self._pack(g, buf[off:off + g.numel()])
                off += g.numel()
            works.append((dist.all_reduce(buf[:n], op=dist.ReduceOp.SUM, group=self.group, async_op=True), bucket, buf))
        for w, bucket, buf in works:
            w.wait()
            off = 0
            for g in bucket:
                self._unpack(buf[off:off + g.numel()], g, 1.0 / world)
                off += g.numel()
