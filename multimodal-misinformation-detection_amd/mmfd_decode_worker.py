"""Decode worker functions of mmfd.hostdecode, in a module of their own that imports neither torch
nor the mmfd package: the decode processes fork from a server that has imported only this module,
numpy and PIL (a server that had imported torch left, once in a few runs, workers that never
exited, hanging their parent's interpreter exit). Loaded by mmfd.hostdecode as the top-level
module `mmfd_decode_worker`."""
from multiprocessing import shared_memory

import numpy as np


def decode_group(paths):
    """worker: decode `paths` -> (shm name or None, [(h, w, byte offset)])"""
    from PIL import Image
    arrs = []
    for p in paths:
        with Image.open(p) as im:
            arrs.append(np.asarray(im.convert("RGB"), dtype=np.uint8))
    total = sum(a.nbytes for a in arrs)
    if total == 0:
        return None, [(a.shape[0], a.shape[1], 0) for a in arrs]
    # (registered with the resource tracker the whole process tree shares; the caller's unlink()
    # unregisters it, and the tracker unlinks it at the end should the caller never get to it)
    shm = shared_memory.SharedMemory(create=True, size=total)
    meta, off = [], 0
    for a in arrs:
        np.frombuffer(shm.buf, dtype=np.uint8, count=a.nbytes, offset=off)[:] = a.reshape(-1)
        meta.append((a.shape[0], a.shape[1], off))
        off += a.nbytes
    name = shm.name
    shm.close()
    return name, meta


_ATTACHED = {}


def decode_group_into(shm_name, base, cap, paths):
    """worker: decode `paths` into the shared ring at [base, base + cap), packed back to back ->
    [(h, w, offset from base)] with offset -1 and the pixels themselves for an image past the space"""
    from PIL import Image
    shm = _ATTACHED.get(shm_name)
    if shm is None:
        shm = _ATTACHED[shm_name] = shared_memory.SharedMemory(name=shm_name)
    out, off = [], 0
    for p in paths:
        with Image.open(p) as im:
            a = np.asarray(im.convert("RGB"), dtype=np.uint8)
        if off + a.nbytes <= cap:
            np.frombuffer(shm.buf, dtype=np.uint8, count=a.nbytes, offset=base + off)[:] = a.reshape(-1)
            out.append((a.shape[0], a.shape[1], off, None))
            off += a.nbytes
        else:
            out.append((a.shape[0], a.shape[1], -1, a))
    return out
