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


class GradAllReduce:
    def __init__(self, bucket_mb: float = 64.0, group=None):
        self.bucket_elems = int(bucket_mb * (1 << 20) / 4)
        self.group = group
        self._bufs = {}

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
                K.cast(g, torch.float32, out=buf[off:off + g.numel()])
                off += g.numel()
            works.append((dist.all_reduce(buf[:n], op=dist.ReduceOp.SUM, group=self.group, async_op=True), bucket, buf))
        for w, bucket, buf in works:
            w.wait()
            off = 0
            for g in bucket:
                K.axpby(1.0 / world, buf[off:off + g.numel()], 0.0, None, out=g)
                off += g.numel()
