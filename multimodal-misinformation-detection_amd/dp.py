"""Data parallelism (BASELINE config 4): one process per GPU, gradients averaged with RCCL over xGMI.

The reference is single-device (train.py:321); the batch dimension shards naturally (independent
claim/evidence pairs), so each rank runs the full step on its own 256 pairs and the only exchange is
the gradient average. The all-reduce is OVERLAPPED with the backward pass: the hand-written
backward of each encoder reports every layer's finished parameter gradients (StepCtx.flush_ready),
they are packed into ~32 MB fp32 buckets and each full bucket is all-reduced asynchronously on
RCCL's stream while the next layers' backward kernels run on the compute stream. `finish()` waits
for the outstanding buckets and writes the averages into the parameters' .grad.

The two encoders run on two HIP streams (mmfd.train.FusionTrainer._encode), and autograd runs each
encoder's backward on its forward's stream, so gradients become ready on two streams. Buckets are
therefore kept per stream: a bucket is packed and handed to RCCL on the stream that produced its
gradients (RCCL orders a collective after the CURRENT stream only), and the per-step order of the
collectives is the host order of the backward calls, the same on every rank.

Graph capture of the DP step (FusionTrainer.capture): the captured all-reduces run on a DEDICATED
process group (`capture_group()`, created with the communicator connected eagerly, so its RCCL
stream never carries an eager collective), and the capture uses the thread-local error mode. Both
are needed for the capture not to depend on timing: ProcessGroupNCCL's watchdog thread polls the
events of every eager collective of a group; in the global capture mode any such query from the
watchdog during a capture is refused (hipErrorStreamCaptureUnsupported), and an event last recorded
on a stream that has since joined a capture is refused as well (hipErrorCapturedEvent) — the two
aborts of round 4. With the eager collectives on the default group's stream and the captured ones
on the capture group's stream, and the watchdog's queries allowed by the thread-local mode, no
query can hit a capturing stream whenever it happens. `consistent()` is the self-check afterwards:
after one replay every rank must hold bitwise-identical gradients and parameters (ranks train on
different batches, so that holds only if the captured all-reduce really ran).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import kernels as K


def state_checksum(tensors) -> torch.Tensor:
    """int64 checksum of the exact bits of `tensors` (None entries skipped), on their device: the
    integer sum of each tensor's words (wrapping, so the order of the additions does not matter)
    times an odd per-position weight — equal tensors in the same order give equal checksums, and a
    tensor that differs in any bit almost never does."""
    acc = None
    for i, t in enumerate(tensors):
        if t is None:
            continue
        t = t.detach().contiguous().reshape(-1)
        words = t.view(torch.int32) if t.element_size() == 4 else t.view(torch.int16) if t.element_size() == 2 \
            else t.view(torch.int64) if t.element_size() == 8 else t.view(torch.uint8)
        s = words.to(torch.int64).sum() * (2 * i + 1)
        acc = s if acc is None else acc + s
    if acc is None:
        acc = torch.zeros((), dtype=torch.int64)
    return acc.reshape(1)


def ranks_agree(value: torch.Tensor, group=None) -> bool:
    """True when `value` (an int64 tensor) is identical on every rank of `group`: its MIN and its
    MAX over the ranks are equal. Every rank gets the same answer."""
    lo, hi = value.clone(), value.clone()
    dist.all_reduce(lo, op=dist.ReduceOp.MIN, group=group)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=group)
    return bool(torch.equal(lo, hi))


def _pack(g, dst):
    K.cast(g, torch.float32, out=dst)


def _unpack(src, g, scale):
    K.axpby(scale, src, 0.0, None, out=g)


class GradAllReduce:
    """`pack(grad, flat_slice)` / `unpack(flat_slice, grad, scale)` default to the HIP cast/axpby
    kernels; they are parameters only so the bucketing + collective logic can be exercised on the
    CPU (gloo) in tests."""

    def __init__(self, bucket_mb: float = 32.0, group=None, pack=_pack, unpack=_unpack, force=False):
        """`force`: run the bucketing, packing and collectives even with one rank (tests and the DP
        overhead measurement on a one-GPU box; a world-size-1 all-reduce leaves the values as they are)"""
        self.bucket_elems = max(1, int(bucket_mb * (1 << 20) / 4))
        self.group = group
        self.force = bool(force)
        self._capture_group = None
        self._bufs = {}
        self._pack, self._unpack = pack, unpack
        self.last_buckets = {}
        self.begin()

    # ---- per-step protocol ------------------------------------------------------------------------
    def begin(self):
        self._pending = {}  # stream key -> [pending (param, grad) list, element count]
        self._works = []
        self._nbucket = {}

    @staticmethod
    def _stream_key(g):
        return torch.cuda.current_stream(g.device).cuda_stream if g.is_cuda else None

    def ready(self, pairs):
        """pairs: iterable of (parameter, finished fp32 gradient tensor), produced on the current stream"""
        if not self._active():
            return
        for p, g in pairs:
            if g is None:
                continue
            key = self._stream_key(g)
            ent = self._pending.setdefault(key, [[], 0])
            ent[0].append((p, g))
            ent[1] += g.numel()
            if ent[1] >= self.bucket_elems:
                self._flush(key)

    def hook_for(self, model):
        """callable(names, grads) for StepCtx.grad_ready: maps parameter names of `model` to params"""
        params = dict(model.named_parameters())
        return lambda names, grads: self.ready((params[n], grads[n]) for n in names if n in params)

    def finish(self):
        """flush, wait, and write the averages into each parameter's .grad (the tensor autograd
        installed, which may or may not be the one that was packed)"""
        if not self._active():
            return
        # leftovers of every stream, packed on the calling stream: backward() has returned, so the
        # calling stream is already ordered after every gradient it reads
        for key in list(self._pending):
            self._flush(key)
        world = dist.get_world_size(self.group)
        for w, items, buf in self._works:
            w.wait()
            off = 0
            for p, g in items:
                n = g.numel()
                self._unpack(buf[off:off + n], p.grad if p.grad is not None else g, 1.0 / world)
                off += n
        self.last_buckets = dict(self._nbucket)  # buckets per stream of the step just finished
        self.begin()

    def broadcast_params(self, params, src=0):
        """Make every rank start from rank `src`'s parameters (called once when a trainer is built:
        ranks may have initialised their replicas from different seeds). Parameters are flattened
        into bucket-sized fp32 buffers, one broadcast per bucket; the copies back are plain
        in-place writes (they bump each parameter's version counter, so the bf16 weight shadows
        are re-cast from the broadcast values)."""
        self.broadcast_tensors(params, src)

    def broadcast_tensors(self, tensors, src=0):
        """rank `src`'s values of `tensors` (fp32, any shapes; None entries skipped) on every rank,
        in bucket-sized broadcasts on `group`"""
        if not self._active():
            return
        params = [p for p in tensors if p is not None]
        i = 0
        while i < len(params):
            j, n = i, 0
            while j < len(params) and (j == i or n + params[j].numel() <= self.bucket_elems):
                n += params[j].numel()
                j += 1
            group = params[i:j]
            buf = torch.empty(n, device=group[0].device, dtype=torch.float32)
            off = 0
            with torch.no_grad():
                for p in group:
                    buf[off:off + p.numel()].copy_(p.detach().reshape(-1))
                    off += p.numel()
                dist.broadcast(buf, src=src, group=self.group)
                off = 0
                for p in group:
                    p.detach().copy_(buf[off:off + p.numel()].view(p.shape))
                    off += p.numel()
            i = j

    def allreduce_grads(self, params):
        """non-overlapped form: average every .grad of `params`"""
        self.begin()
        self.ready((p, p.grad) for p in params)
        self.finish()

    # ---- graph capture -------------------------------------------------------------------------------
    def capture_group(self):
        """The process group the captured step's all-reduces run on (collective: every rank calls it
        at the same point; created once — FusionTrainer.capture calls it BEFORE its eager warm-up
        steps, so a rank that fails later cannot leave the others waiting inside new_group). Same
        ranks as `group`; with a device-bound default group (init_process_group(device_id=...), as
        bench.py and train.py do) its communicator is connected at creation, so no collective ever
        runs on it outside a capture. An RCCL default group WITHOUT a bound device would connect the
        new communicator lazily — inside the capture — so that case is refused (every rank raises
        the same error before any collective; capture_dp_step then runs eager steps)."""
        if self._capture_group is None:
            if dist.get_backend(self.group) == "nccl":
                from torch.distributed import distributed_c10d as c10d
                if getattr(c10d._get_default_group(), "bound_device_id", None) is None:
                    raise RuntimeError("mmfd DP capture needs a device-bound default process group "
                                       "(init_process_group(..., device_id=torch.device('cuda', local_rank)))")
            ranks = None if self.group is None else dist.get_process_group_ranks(self.group)
            self._capture_group = dist.new_group(ranks=ranks, group_desc="mmfd_dp_capture")
        return self._capture_group

    def use_capture_group(self, on: bool = True):
        """route this object's collectives to capture_group() (on) or back to `group` (off)"""
        self._use_capture = bool(on)
        if on:
            self.capture_group()

    def consistent(self, tensors) -> bool:
        """Cross-rank self-check: True when every rank holds bitwise-identical `tensors` (gradients
        and parameters after a data-parallel step); every rank gets the same answer. Runs eager
        collectives on `group`."""
        if not dist.is_initialized():
            return True
        c = state_checksum(tensors)
        return ranks_agree(c, self.group)

    # ---- internals -----------------------------------------------------------------------------------
    def _coll_group(self):
        return self._capture_group if getattr(self, "_use_capture", False) else self.group

    def _active(self):
        return dist.is_initialized() and (self.force or dist.get_world_size(self.group) > 1)

    def _flush(self, key):
        items, n = self._pending.pop(key, [[], 0])
        if not items:
            return
        i = self._nbucket.get(key, 0)
        self._nbucket[key] = i + 1
        dev = items[0][1].device
        buf = self._bufs.get((key, i))
        if buf is None or buf.numel() < n or buf.device != dev:
            buf = self._bufs[(key, i)] = torch.empty(max(n, self.bucket_elems), device=dev, dtype=torch.float32)
        off = 0
        for _, g in items:
            self._pack(g, buf[off:off + g.numel()])
            off += g.numel()
        work = dist.all_reduce(buf[:n], op=dist.ReduceOp.SUM, group=self._coll_group(), async_op=True)
        self._works.append((work, items, buf))
