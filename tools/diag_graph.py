"""Staged HIP-graph capture checks (one process; stops at the first failure): a captured GEMM, a
captured zero fill, a head-only training step, the tiny full training step."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import mmfd  # noqa: E402,F401
from mmfd import kernels as K  # noqa: E402


def log(*a):
    print(*a, flush=True)


def stage_gemm():
    A = torch.randn(300, 96, device="cuda")
    W = torch.randn(80, 96, device="cuda")
    out = torch.empty(300, 80, device="cuda")
    ref = K.gemm(A, W)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        K.gemm(A, W, out=out)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        K.gemm(A, W, out=out)
    out.zero_()
    g.replay()
    torch.cuda.synchronize()
    log("gemm graph ok", torch.equal(out, ref))


def stage_zero():
    z = torch.ones(1000, device="cuda")
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        K.zero_(z)
    g.replay()
    torch.cuda.synchronize()
    log("zero graph ok", float(z.abs().sum()))


def stage_head():
    from mmfd.model import MisinformationDetectionModel
    from mmfd.train import FusionTrainer
    torch.manual_seed(0)
    head = MisinformationDetectionModel(48, 40, 32, 4, dropout=0.1, hidden_dim=16).cuda()
    tr = FusionTrainer(None, None, head, lr=1e-3, precision="fp32")
    g = torch.Generator().manual_seed(1)
    b = {"claim_text_embeds": torch.randn(2, 8, 48, generator=g).cuda(),
         "doc_text_embeds": torch.randn(2, 9, 48, generator=g).cuda(),
         "claim_image_embeds": torch.randn(2, 13, 40, generator=g).cuda(),
         "doc_image_embeds": torch.randn(2, 11, 40, generator=g).cuda(),
         "labels": torch.randint(0, 3, (2, 4), generator=g).cuda()}
    tr.capture(b, warmup=2)
    log("head captured")
    for _ in range(3):
        tr.replay()
    torch.cuda.synchronize()
    log("head graph ok", tr.replay().tolist())


def _head_setup(dropout=0.1):
    from mmfd.model import MisinformationDetectionModel
    torch.manual_seed(0)
    head = MisinformationDetectionModel(48, 40, 32, 4, dropout=dropout, hidden_dim=16).cuda()
    g = torch.Generator().manual_seed(1)
    X = [torch.randn(2, n, d, generator=g).cuda() for n, d in ((8, 48), (13, 40), (9, 48), (11, 40))]
    labels = torch.randint(0, 3, (2, 4), generator=g).cuda()
    return head, X, labels


def _cap(fn, warm=2, prep=None):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(warm):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    if prep is not None:
        prep()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = fn()
    return g, out


def stage_h1():  # forward only, eval, no grad
    head, X, _ = _head_setup()
    head.eval()
    with torch.no_grad():
        g, out = _cap(lambda: head(*X))
    g.replay()
    torch.cuda.synchronize()
    log("h1 ok")


def stage_h2():  # forward (train, dropout) + loss, no grad
    from mmfd.train import path_losses
    head, X, labels = _head_setup()
    with torch.no_grad():
        g, out = _cap(lambda: path_losses(head(*X), labels))
    g.replay()
    torch.cuda.synchronize()
    log("h2 ok", out.tolist())


def stage_h3():  # forward + backward, no optimizer
    from mmfd.train import path_losses
    head, X, labels = _head_setup()
    gv = torch.tensor([1.0, 0, 0, 0, 0], device="cuda")

    def fb():
        for p in head.parameters():
            p.grad = None
        loss = path_losses(head(*X), labels)
        torch.autograd.backward(loss, gv)
        return loss
    g, out = _cap(fb)
    g.replay()
    torch.cuda.synchronize()
    log("h3 ok", out.tolist())


def stage_h4():  # h3 + dropout off
    from mmfd.train import path_losses
    head, X, labels = _head_setup(dropout=0.0)
    gv = torch.tensor([1.0, 0, 0, 0, 0], device="cuda")

    def fb():
        for p in head.parameters():
            p.grad = None
        loss = path_losses(head(*X), labels)
        torch.autograd.backward(loss, gv)
        return loss
    g, out = _cap(fb)
    g.replay()
    torch.cuda.synchronize()
    log("h4 ok", out.tolist())


def stage_h5():  # h3 + mmfd AdamW (late-bound capture table)
    from mmfd.optim import AdamW
    from mmfd.train import path_losses
    head, X, labels = _head_setup()
    opt = AdamW(head.parameters(), lr=1e-3)
    gv = torch.tensor([1.0, 0, 0, 0, 0], device="cuda")

    def fb():
        for p in head.parameters():
            p.grad = None
        loss = path_losses(head(*X), labels)
        torch.autograd.backward(loss, gv)
        opt.step()
        return loss
    g, out = _cap(fb, prep=opt.prepare_capture)
    opt.finalize_capture()
    g.replay()
    torch.cuda.synchronize()
    log("h5 ok", out.tolist())


def stage_h6():  # FusionTrainer step with the optimizer step disabled
    from mmfd.model import MisinformationDetectionModel
    from mmfd.train import FusionTrainer
    torch.manual_seed(0)
    head = MisinformationDetectionModel(48, 40, 32, 4, dropout=0.1, hidden_dim=16).cuda()
    tr = FusionTrainer(None, None, head, lr=1e-3, precision="fp32")
    tr.optimizer.step = lambda *a, **k: None
    g = torch.Generator().manual_seed(1)
    b = {"claim_text_embeds": torch.randn(2, 8, 48, generator=g).cuda(),
         "doc_text_embeds": torch.randn(2, 9, 48, generator=g).cuda(),
         "claim_image_embeds": torch.randn(2, 13, 40, generator=g).cuda(),
         "doc_image_embeds": torch.randn(2, 11, 40, generator=g).cuda(),
         "labels": torch.randint(0, 3, (2, 4), generator=g).cuda()}
    tr.capture(b, warmup=2)
    log("h6 captured")
    tr.replay()
    torch.cuda.synchronize()
    log("h6 ok", tr.replay().tolist())


def stage_h7():  # h5, but check the late-bound table against the live tensors before any replay
    import ctypes
    from mmfd.optim import AdamW
    from mmfd.train import path_losses
    head, X, labels = _head_setup()
    opt = AdamW(head.parameters(), lr=1e-3)
    gv = torch.tensor([1.0, 0, 0, 0, 0], device="cuda")

    def fb():
        for p in head.parameters():
            p.grad = None
        loss = path_losses(head(*X), labels)
        torch.autograd.backward(loss, gv)
        opt.step()
        return loss
    g, out = _cap(fb, prep=opt.prepare_capture)
    pend = list(opt._pending_capture)
    opt.finalize_capture()
    torch.cuda.synchronize()
    bad = 0
    for t, entries in pend:
        raw = bytes(t.cpu().numpy().tobytes())
        arr = (K.AdamWTensor * len(entries)).from_buffer_copy(raw)
        for i, (p, gr, m, v, st) in enumerate(entries):
            a = arr[i]
            live = (p.data_ptr(), p.grad.data_ptr() if p.grad is not None else 0, m.data_ptr(), v.data_ptr(),
                    st.data_ptr(), p.numel())
            tab = (a.param, a.grad, a.exp_avg, a.exp_avg_sq, a.step, a.numel)
            if live != tab or gr.data_ptr() != live[1]:
                bad += 1
                log("MISMATCH", i, tuple(p.shape), live, tab, gr.data_ptr(), st.device, st.dtype, st.shape)
    log("table entries checked, bad =", bad, "tables", len(pend))
    if bad:
        return
    n = len(pend[0][1])
    K.adamw(pend[0][0], n, max(e[0].numel() for e in pend[0][1]), 1e-3, 0.9, 0.999, 1e-8, 1e-2)
    torch.cuda.synchronize()
    log("eager launch on the captured table ok")


def stage_h8():  # only the AdamW step captured (gradients computed eagerly and kept)
    from mmfd.optim import AdamW
    head, X, labels = _head_setup()
    opt = AdamW(head.parameters(), lr=1e-3)
    for p in head.parameters():
        p.grad = torch.randn_like(p)
    g, _ = _cap(lambda: opt.step(), prep=opt.prepare_capture)
    opt.finalize_capture()
    torch.cuda.synchronize()
    log("h8 captured")
    g.replay()
    torch.cuda.synchronize()
    log("h8 ok")


def stage_cmp(precision="fp32"):  # captured vs eager steps: max differences
    from tests.smoke_impl import build_pair, tiny_batch
    tr_e, _ = build_pair(precision, dropout=0.1)
    tr_g, _ = build_pair(precision, dropout=0.1)
    b1 = {k: v.cuda() for k, v in tiny_batch(3, seed=41).items()}
    b2 = {k: v.cuda() for k, v in tiny_batch(3, seed=42).items()}
    tr_g.capture({k: v.clone() for k, v in b1.items()}, warmup=2)
    le = [tr_e.step(b1) for _ in range(2)]
    torch.cuda.synchronize()
    for m_e, m_g in ((tr_e.text_encoder, tr_g.text_encoder), (tr_e.image_encoder, tr_g.image_encoder),
                     (tr_e.head, tr_g.head)):
        d = max((p - q).abs().max().item() for p, q in zip(m_e.parameters(), m_g.parameters()))
        log("after warmup: param max diff", type(m_e).__name__, d)
    le += [tr_e.step(b1), tr_e.step(b2), tr_e.step(b1)]
    lg = [tr_g.replay().clone(), tr_g.replay(b2).clone(), tr_g.replay(b1).clone()]
    torch.cuda.synchronize()
    for a, b in zip(le[2:], lg):
        log("loss diff", (a - b).abs().max().item(), a.tolist())
    for m_e, m_g in ((tr_e.text_encoder, tr_g.text_encoder), (tr_e.image_encoder, tr_g.image_encoder),
                     (tr_e.head, tr_g.head)):
        worst = max(((p - q).abs().max().item(), n) for (n, p), (_, q) in zip(m_e.named_parameters(), m_g.named_parameters()))
        log("param max diff", type(m_e).__name__, worst)


def stage_full():
    from tests.smoke_impl import build_pair, tiny_batch
    tr, _ = build_pair("fp32", dropout=0.1)
    b = {k: v.cuda() for k, v in tiny_batch(3, seed=41).items()}
    tr.capture(b, warmup=2)
    log("full captured")
    for _ in range(3):
        tr.replay()
    torch.cuda.synchronize()
    log("full graph ok", tr.replay().tolist())


if __name__ == "__main__":
    K.load()
    for st in sys.argv[1:] or ["gemm", "zero", "head", "full"]:
        log("stage", st)
        globals()["stage_" + st]()
        torch.cuda.synchronize()
    log("ALL OK")
