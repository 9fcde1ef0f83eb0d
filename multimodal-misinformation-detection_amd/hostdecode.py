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
from multiprocessing import resource_tracker, shared_memory

import numpy as np


def _decode_group(paths):
    """worker: decode `paths` -> (shm name or None, [(h, w, byte offset)])"""
    from PIL import Image
    arrs = []
    for p in paths:
        with Image.open(p) as im:
            arrs.append(np.asarray(im.convert("RGB"), dtype=np.uint8))
    total = sum(a.nbytes for a in arrs)
    if total == 0:
        return None, [(a.shape[0], a.shape[1], 0) for a in arrs]
    shm = shared_memory.SharedMemory(create=True, size=total)
    # the caller owns (and unlinks) the block: keep this process's resource tracker out of it
    resource_tracker.unregister(shm._name, "shared_memory")
    meta, off = [], 0
    for a in arrs:
        np.frombuffer(shm.buf, dtype=np.uint8, count=a.nbytes, offset=off)[:] = a.reshape(-1)
        meta.append((a.shape[0], a.shape[1], off))
        off += a.nbytes
    name = shm.name
    shm.close()
    return name, meta


class DecodePool:
    """`submit(paths)` -> handle; `get(handle)` -> (list of uint8 HxWx3 arrays, release callable)."""

    def __init__(self, workers=None, group=8):
        import concurrent.futures as cf
        import multiprocessing as mp
        self.workers = int(workers or min(16, len(os.sched_getaffinity(0))))
        self.group = max(1, int(group))
        ctx = mp.get_context("forkserver")
        # the workers fork from a server that imported this module (and numpy / PIL) once
        ctx.set_forkserver_preload([__name__, "PIL.Image"])
        self._ex = cf.ProcessPoolExecutor(max_workers=self.workers, mp_context=ctx)

    def submit(self, paths):
        paths = list(paths)
        return [self._ex.submit(_decode_group, paths[i:i + self.group]) for i in range(0, len(paths), self.group)]

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
            resource_tracker.unregister(shm._name, "shared_memory")  # attached, not created here
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
        self._ex.shutdown(wait=True, cancel_futures=True)

    def __del__(self):
        try:
            self._ex.shutdown(wait=False, cancel_futures=True)
        except Exception:
            pass
