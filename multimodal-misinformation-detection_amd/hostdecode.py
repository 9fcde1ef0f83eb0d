"""Host image decode off the GIL, for the config-5 corpus build (im2im_retrieval.py:69-78 opens every
image with PIL in the calling process).

PIL releases the GIL inside the JPEG decoder but not around file parsing and `convert("RGB")`, so a
thread pool saturates near 1.6k images/s. `DecodePool` decodes in a pool of
worker PROCESSES (forkserver: nothing is forked from a process that has initialised the GPU). A task
is a group of paths; the worker decodes each with exactly the calls of `evidence._decode`
(Image.open(path).convert("RGB") -> uint8 HWC, the same bytes), packs the group into one POSIX
shared-memory block and returns only its name and the image shapes; the caller copies the block
out in one memcpy and unlinks it — no pickled pixels cross a pipe, and the main process's only
per-image work is that copy and the GPU preprocessing's copy into its pinned upload buffer.
"""
from __future__ import annotations

import os
import sys
from multiprocessing import shared_memory
from multiprocessing import util as mp_util

import numpy as np

# the worker functions live in a torch-free top-level module (see mmfd_decode_worker.py)
_PKG_DIR = os.path.dirname(os.path.abspath(__file__))
if _PKG_DIR not in sys.path:
    sys.path.append(_PKG_DIR)
import mmfd_decode_worker as _dw  # noqa: E402


def _shutdown_executor(ex):
    ex.shutdown(wait=True, cancel_futures=True)


class DecodePool:
    """`submit(paths)` -> handle; `get(handle)` -> (list of uint8 HxWx3 arrays, release callable)."""

    def __init__(self, workers=None, group=8):
        import concurrent.futures as cf
        import multiprocessing as mp
        self.workers = int(workers or min(16, len(os.sched_getaffinity(0))))
        self.group = max(1, int(group))
        ctx = mp.get_context("forkserver")
        # the workers fork from a server that imported this module (and numpy / PIL) once
        ctx.set_forkserver_preload(["mmfd_decode_worker", "PIL.Image"])
        self._ex = cf.ProcessPoolExecutor(max_workers=self.workers, mp_context=ctx)
        # shut the workers down before the process's exit joins its children: in a multiprocessing
        # child (a corpus-build rank) the exit joins them before concurrent.futures' own exit hook
        # has told them to stop — a hang whenever the pool was still alive at that point
        self._fin = mp_util.Finalize(self, _shutdown_executor, args=(self._ex,), exitpriority=10)

    def submit(self, paths):
        paths = list(paths)
        return [self._ex.submit(_dw.decode_group, paths[i:i + self.group]) for i in range(0, len(paths), self.group)]

    @staticmethod
    def get(handle):
        """-> (list of uint8 HxWx3 arrays in submission order, release callable). Each group's block
        is copied out of shared memory in one memcpy and unlinked here, so nothing outlives the call
        (a zero-copy mapping would pin the block to whatever still references a view)."""
        out = []
        for fut in handle:
            name, meta = fut.result()
            if name is None:
                out += [np.zeros((h, w, 3), np.uint8) for h, w, _ in meta]
                continue
            shm = shared_memory.SharedMemory(name=name)
            try:
                src = np.frombuffer(shm.buf, dtype=np.uint8)
                block = src.copy()
                del src
            finally:
                shm.close()
                shm.unlink()
            for h, w, off in meta:
                out.append(block[off:off + h * w * 3].reshape(h, w, 3))
        return out, (lambda: None)

    def close(self):
        self._fin()  # (runs once)


# ---- decode straight into page-locked shared memory (no host copies in the caller) -------------------
class RingUnavailable(RuntimeError):
    """the page-locked shared-memory ring cannot be set up on this host"""


def _release_ring(ex, shm, addr, device):
    ex.shutdown(wait=True, cancel_futures=True)
    try:
        import torch
        torch.cuda.synchronize(device)  # the uploads out of the ring have run
        torch._C._cudart.cudaHostUnregister(addr)
    except Exception:  # (at interpreter exit the HIP runtime may already be gone)
        pass
    try:
        shm.close()
    except BufferError:  # a view still alive: the mapping goes with the process
        pass
    shm.unlink()


class PinnedDecodeRing:
    """Host decode for the GPU corpus build without host-side copies: a POSIX shared-memory ring,
    page-locked for the HIP runtime once (hipHostRegister through torch's cudart binding), that the
    decode worker processes write into directly. `submit(paths, slot)` starts decoding one batch into
    ring slot `slot` (groups of `group` images, `cap` bytes per image on average per group, packed);
    `upload(handle, slot)` issues the asynchronous host->device copies of the batch's pixels and
    returns (device uint8 buffer, [(h, w)], [byte offsets]); the slot is reused only after the
    stream has consumed its copies (an event per slot). Images that do not fit their group's space
    come back through the pipe and are uploaded from ordinary memory."""

    def __init__(self, batch, device, workers=None, group=8, cap=None, slots=2):
        """`cap`: ring bytes per image (default env MMFD_DECODE_RING_CAP or 1 MiB — a 512x512 RGB
        image is 0.75 MiB; larger images come back through the pipe). The ring is slots x batch x cap
        bytes of /dev/shm, page-locked: raises RingUnavailable when the shared memory or the page
        locking cannot be had (the caller then decodes with the process pool or threads)."""
        import concurrent.futures as cf
        import ctypes
        import multiprocessing as mp

        import torch
        if cap is None:
            cap = int(os.environ.get("MMFD_DECODE_RING_CAP", 1 << 20))
        self.device = torch.device(device)
        self.workers = int(workers or min(16, len(os.sched_getaffinity(0))))
        self.group, self.slots = max(1, int(group)), int(slots)
        self.gbytes = self.group * int(cap)
        self.gps = (int(batch) + self.group - 1) // self.group
        self.sbytes = self.gps * self.gbytes
        try:
            self.shm = shared_memory.SharedMemory(create=True, size=self.slots * self.sbytes)
        except OSError as e:  # e.g. a small /dev/shm in a container
            raise RingUnavailable(f"decode ring: {self.slots * self.sbytes} B of shared memory: {e}") from e
        self._addr = ctypes.addressof(ctypes.c_char.from_buffer(self.shm.buf))
        rc = torch._C._cudart.cudaHostRegister(self._addr, self.slots * self.sbytes, 0)
        if int(rc) != 0:
            self.shm.close()
            self.shm.unlink()
            raise RingUnavailable(f"hipHostRegister of the decode ring failed ({rc})")
        self.host = torch.frombuffer(self.shm.buf, dtype=torch.uint8)
        self._events = [None] * self.slots
        self._writers = [None] * self.slots  # the decode futures that write into each slot
        ctx = mp.get_context("forkserver")
        ctx.set_forkserver_preload(["mmfd_decode_worker", "PIL.Image"])
        self._ex = cf.ProcessPoolExecutor(max_workers=self.workers, mp_context=ctx)
        # (see DecodePool: the workers stop and the ring is released before the process exit joins
        # its children)
        self._fin = mp_util.Finalize(self, _release_ring, args=(self._ex, self.shm, self._addr, self.device),
                                     exitpriority=10)

    def submit(self, paths, slot):
        import concurrent.futures as cf
        prev = self._writers[slot]
        if prev is not None:
            # every decode task that writes this slot has finished — also when its batch was never
            # uploaded (a build that stopped between submit and upload): no stale write can land
            # after the new batch's
            cf.wait(prev)
            self._writers[slot] = None
        ev = self._events[slot]
        if ev is not None:
            ev.synchronize()  # the previous batch's copies out of this slot have run
            self._events[slot] = None
        paths = list(paths)
        if len(paths) > self.gps * self.group:
            raise ValueError("batch larger than the ring slot")
        handle = [self._ex.submit(_dw.decode_group_into, self.shm.name, slot * self.sbytes + gi * self.gbytes,
                                  self.gbytes, paths[i:i + self.group])
                  for gi, i in enumerate(range(0, len(paths), self.group))]
        self._writers[slot] = handle
        return handle

    def upload(self, handle, slot):
        import torch
        res = [f.result() for f in handle]
        shapes, offs, spans, extra, total = [], [], [], [], 0
        for gi, items in enumerate(res):
            used = 0
            for h, w, off, arr in items:
                shapes.append((h, w))
                if off >= 0:
                    offs.append(None)  # filled below: the group's bytes land contiguously
                    used = max(used, off + h * w * 3)
                else:
                    offs.append(None)
                    extra.append((len(shapes) - 1, arr))
            spans.append((gi, used))
        dsrc = torch.empty(max(1, sum(u for _, u in spans) + sum(a.nbytes for _, a in extra)), dtype=torch.uint8,
                           device=self.device)
        k, pos = 0, 0
        for (gi, used), items in zip(spans, res):
            base = slot * self.sbytes + gi * self.gbytes
            if used:
                dsrc[pos:pos + used].copy_(self.host[base:base + used], non_blocking=True)
            for h, w, off, arr in items:
                if off >= 0:
                    offs[k] = pos + off
                k += 1
            pos += used
        for i, arr in extra:
            dsrc[pos:pos + arr.nbytes].copy_(torch.from_numpy(arr.reshape(-1)))
            offs[i] = pos
            pos += arr.nbytes
        ev = torch.cuda.Event()
        ev.record()
        self._events[slot] = ev
        return dsrc, shapes, offs

    def close(self):
        self.host = None  # (the view would pin the mapping)
        self._fin()  # (runs once)
