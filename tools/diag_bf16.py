"""bf16 vs oracle diagnostics: head-only (config 1 dims) with/without dropout; whole step tiny."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import mmfd  # noqa
from mmfd.model import MisinformationDetectionModel
from mmfd.train import path_losses
from mmfd.dataset import LABEL_TABLE
from oracle import fusion_head as OF
from oracle.dropout_hash import make_drop
from tests.smoke_impl import TINY, FULL, build_pair, compare_step, tiny_batch


def head(prec, p, Lt=512, Li=64, dt=384, di=1024, B=4):
    g = torch.Generator().manual_seed(11)
    X = [torch.randn(B, Lt, dt, generator=g), torch.randn(B, Li, di, generator=g),
         torch.randn(B, Lt, dt, generator=g), torch.randn(B, Li, di, generator=g)]
    cat = torch.randint(0, 5, (B,), generator=g)
    m = MisinformationDetectionModel(dt, di, 256, 8, dropout=p, hidden_dim=64).cuda().train().set_precision(prec)
    m.manual_seed(777)
    P = {n: q.detach().cpu().clone().requires_grad_(True) for n, q in m.named_parameters()}
    out = m(*(x.cuda() for x in X))
    ref = OF.model_forward(P, *X, num_heads=8, drop=make_drop(777, p) if p > 0 else None)
    lab = LABEL_TABLE[cat]
    loss = path_losses(out, lab.cuda())
    tot, _ = OF.path_loss(ref, lab)
    loss[0].backward()
    tot.backward()
    torch.cuda.synchronize()
    yerr = max((y.detach().float().cpu() - r.detach()).abs().max().item() for a, b in zip(out, ref) for y, r in zip(a, b))
    res = []
    for n, q in m.named_parameters():
        r = P[n].grad
        if r is None:
            continue
        d = q.grad.double().cpu() - r.double()
        res.append((d.abs().max().item() / r.abs().max().item(), d.norm().item() / r.double().norm().item(), n))
    res.sort(reverse=True)
    print(f"head {prec} p={p} L={Lt}/{Li}: logits {yerr:.3e} loss {abs(loss[0].item()-tot.item()):.3e}")
    for e in res[:5]:
        print("   %.3e %.3e %s" % e)


for prec in ("bf16",):
    for p in (0.0, 0.1):
        head(prec, p)
        head(prec, p, Lt=128, Li=197, dt=768, di=768)
for p in (0.0, 0.1):
    tr, ref = build_pair("bf16", dropout=p)
    rep = []
    l, w = compare_step(tr, ref, tiny_batch(3, seed=4), loss_tol=1e9, grad_rtol=1e9, report=rep)
    print(f"tiny step bf16 p={p}: loss {l:.3e} worst {w:.3e}")
    for k, e, en in sorted(rep, key=lambda t: -t[1])[:5]:
        print(f"   {e:.3e} {en:.3e} {k}")
for p in (0.0, 0.1):
    tr, ref = build_pair("bf16", dropout=p, cfg=FULL, lr=1e-4)
    rep = []
    l, w = compare_step(tr, ref, tiny_batch(2, cfg=FULL, seed=41), loss_tol=1e9, grad_rtol=1e9, report=rep)
    print(f"full step bf16 p={p}: loss {l:.3e} worst {w:.3e}")
    for k, e, en in sorted(rep, key=lambda t: -t[1])[:8]:
        print(f"   {e:.3e} {en:.3e} {k}")
    del tr, ref
