"""Drop-in for `torch.optim.AdamW` (train.py:8, 356, 188) backed by one multi-tensor HIP launch.

Same math as torch's AdamW (decoupled weight decay, bias correction with a per-parameter step),
same state keys ('step', 'exp_avg', 'exp_avg_sq'); parameters whose .grad is None are skipped,
exactly like torch (the reference's `text_self_ln2` / `image_self_ln2` never receive gradients).
The pointer table is cached, so a step can be captured in a hipGraph once warmed up.
"""
from __future__ import annotations

import ctypes

import torch

from . import kernels as K


def _adopt_state(st, p):
    """State loaded from a checkpoint (torch.optim.AdamW's `optimizer_state_dict`, or an mmfd one
    loaded with map_location='cpu') may hold CPU tensors, a python-number / int step or
    non-contiguous moments: the kernel reads raw device pointers, so move every entry onto the
    parameter's device as contiguous fp32 (torch keeps a non-capturable 'step' on the CPU)."""
    step = st.get("step", 0)
    if not torch.is_tensor(step):
        step = torch.tensor(float(step))
    if step.device != p.device or step.dtype != torch.float32 or step.dim() != 0:
        st["step"] = step.detach().reshape(()).to(device=p.device, dtype=torch.float32)
    for k in ("exp_avg", "exp_avg_sq"):
        t = st.get(k)
        if t is None:
            st[k] = torch.zeros_like(p, memory_format=torch.contiguous_format)
            continue
        if tuple(t.shape) != tuple(p.shape):
            raise ValueError(f"AdamW state '{k}' has shape {tuple(t.shape)}, parameter {tuple(p.shape)}")
        if t.device != p.device or t.dtype != torch.float32 or not t.is_contiguous():
            st[k] = t.detach().to(device=p.device, dtype=torch.float32).contiguous()


class AdamW(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2):
        if lr < 0 or eps < 0 or not (0 <= betas[0] < 1 and 0 <= betas[1] < 1) or weight_decay < 0:
            raise ValueError("invalid AdamW hyper-parameters")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self._tables = {}

    def _table(self, entries, device):
        from .blocks import live_shadow
        shadows = []
        for p, *_ in entries:  # the bf16 weight copies the HIP modules read (refreshed in the same launch)
            sh = live_shadow(p.data_ptr())
            ok = sh is not None and sh[0].dtype == torch.bfloat16 and sh[0].numel() == p.numel()
            shadows.append(sh[0].data_ptr() if ok else 0)
        key = tuple((p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), s.data_ptr(), p.numel(), sp)
                    for (p, g, m, v, s), sp in zip(entries, shadows))
        t = self._tables.get(key)
        if t is None:
            arr = (K.AdamWTensor * len(entries))()
            for i, ((p, g, m, v, s), sp) in enumerate(zip(entries, shadows)):
                arr[i].param, arr[i].grad = p.data_ptr(), g.data_ptr()
                arr[i].exp_avg, arr[i].exp_avg_sq = m.data_ptr(), v.data_ptr()
                arr[i].param_bf16 = sp or None
                arr[i].step = s.data_ptr()
                arr[i].numel = p.numel()
            host = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8)
            t = host.to(device)
            self._tables[key] = t
        return t

    # ---- HIP-graph capture: the pointer table is late-bound ------------------------------------------
    # Under stream capture the gradients are fresh graph-pool tensors whose table cannot be uploaded
    # from the host (no synchronous copies while capturing). The captured launch reads a device table
    # that prepare_capture() reserved BEFORE the capture: a table allocated inside the capture would
    # come from the graph's private pool, where it may share bytes with temporaries that earlier
    # kernels of the same graph write at every replay (the host-written pointers would be clobbered
    # before the AdamW launch reads them). finalize_capture() fills the reserved tables once the
    # captured step has assigned every .grad (the same tensors every replay writes).
    def prepare_capture(self):
        dev = next(p.device for g in self.param_groups for p in g["params"])
        self._reserved = [torch.empty(max(1, len(g["params"])) * ctypes.sizeof(K.AdamWTensor), dtype=torch.uint8,
                                      device=dev) for g in self.param_groups]
        self._pending_capture = []

    def _capture_table(self, gi, entries):
        res = getattr(self, "_reserved", None)
        if res is None:
            raise RuntimeError("mmfd AdamW: call prepare_capture() before capturing a step in a HIP graph")
        t = res[gi]
        if t.numel() < len(entries) * ctypes.sizeof(K.AdamWTensor):
            raise RuntimeError("mmfd AdamW: reserved capture table too small")
        self._pending_capture = getattr(self, "_pending_capture", []) + [(t, entries)]
        return t

    @torch.no_grad()
    def finalize_capture(self):
        from .blocks import live_shadow
        for t, entries in getattr(self, "_pending_capture", []):
            arr = (K.AdamWTensor * len(entries))()
            for i, (p, g, m, v, st) in enumerate(entries):
                sh = live_shadow(p.data_ptr())
                ok = sh is not None and sh[0].dtype == torch.bfloat16 and sh[0].numel() == p.numel()
                arr[i].param, arr[i].grad = p.data_ptr(), g.data_ptr()
                arr[i].exp_avg, arr[i].exp_avg_sq = m.data_ptr(), v.data_ptr()
                arr[i].param_bf16 = sh[0].data_ptr() if ok else None
                arr[i].step, arr[i].numel = st.data_ptr(), p.numel()
            t[: ctypes.sizeof(arr)].copy_(torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8))
        # the captured launches read these tables at every replay: keep them alive with the graph
        self._captured_tables = getattr(self, "_captured_tables", []) + [t for t, _ in self._pending_capture]
        self._pending_capture = []
        self._reserved = None

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for gi, group in enumerate(self.param_groups):
            entries = []
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.dtype != torch.float32 or p.grad.dtype != torch.float32:
                    raise TypeError("mmfd AdamW keeps fp32 master parameters and gradients")
                if not (p.is_contiguous() and p.grad.is_contiguous()):
                    raise ValueError("mmfd AdamW needs contiguous params/grads")
                st = self.state[p]
                if not st:
                    st["step"] = torch.zeros((), dtype=torch.float32, device=p.device)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                else:
                    _adopt_state(st, p)
                entries.append((p, p.grad, st["exp_avg"], st["exp_avg_sq"], st["step"]))
            if not entries:
                continue
            b1, b2 = group["betas"]
            if torch.cuda.is_current_stream_capturing():
                table = self._capture_table(gi, entries)
            else:
                table = self._table(entries, entries[0][0].device)
            K.adamw(table, len(entries), max(e[0].numel() for e in entries), group["lr"], b1, b2, group["eps"],
                    group["weight_decay"])
        return loss
