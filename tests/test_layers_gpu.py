"""Standalone drop-in layers (mmfd.layers.MLP / MultiHeadAttention = src/model/layers.py:5-58) on
the HIP path vs the oracle (oracle/fusion_head.py mlp / mha), eval and train mode with identical
counter-hash dropout masks (site "<name>.h" / "<name>.out" / "<name>.attn", seed = manual_seed).
Tolerance (fp32): outputs 1e-5 abs, gradients 1e-5 relative to the tensor's max."""
import pytest
import torch

from mmfd.layers import MLP, MultiHeadAttention
from oracle import fusion_head as OF
from oracle.dropout_hash import make_drop

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _close(a, b, tol):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    assert a.shape == b.shape
    err = (a - b).abs().max().item()
    assert err <= tol * max(1.0, b.abs().max().item()), err


@pytest.mark.parametrize("train", [False, True])
def test_mlp_matches_oracle(train):
    torch.manual_seed(0)
    m = MLP(64, 4.0, dropout=0.1, name="probe_mlp").to(DEV).train(train).manual_seed(77)
    x = torch.randn(3, 11, 64)
    xg = x.to(DEV).requires_grad_(True)
    xr = x.clone().requires_grad_(True)
    P = {"m." + k: v.detach().cpu().clone().requires_grad_(True) for k, v in m.named_parameters()}
    y = m(xg)
    yr = OF.mlp(P, "m", xr, drop=make_drop(77, 0.1) if train else None, site="probe_mlp")
    _close(y, yr, 1e-5)
    R = torch.randn(y.shape)
    (y * R.to(DEV)).sum().backward()
    (yr * R).sum().backward()
    _close(xg.grad, xr.grad, 1e-5)
    for k, p in m.named_parameters():
        _close(p.grad, P["m." + k].grad, 1e-5)


@pytest.mark.parametrize("train", [False, True])
def test_multihead_attention_matches_oracle(train):
    torch.manual_seed(1)
    mha = MultiHeadAttention(64, 2, dropout=0.1, name="probe_mha").to(DEV).train(train).manual_seed(5)
    out = torch.nn.Linear(64, 64).to(DEV)
    Q, Kt, V = (torch.randn(2, n, 64) for n in (9, 13, 13))
    g = [t.to(DEV).requires_grad_(True) for t in (Q, Kt, V)]
    r = [t.clone().requires_grad_(True) for t in (Q, Kt, V)]
    P = {"o.weight": out.weight.detach().cpu().clone().requires_grad_(True),
         "o.bias": out.bias.detach().cpu().clone().requires_grad_(True)}
    y = mha(*g, out)
    yr = OF.mha(*r, P, "o", 2, drop=make_drop(5, 0.1) if train else None, site="probe_mha")
    _close(y, yr, 1e-5)
    R = torch.randn(y.shape)
    (y * R.to(DEV)).sum().backward()
    (yr * R).sum().backward()
    for a, b in zip(g, r):
        _close(a.grad, b.grad, 1e-5)
    _close(out.weight.grad, P["o.weight"].grad, 1e-5)
    _close(out.bias.grad, P["o.bias"].grad, 1e-5)


def test_standalone_dropout_is_reproducible_and_advances():
    torch.manual_seed(2)
    a = MLP(32, 2.0, dropout=0.5, name="rep").to(DEV).train().manual_seed(9)
    b = MLP(32, 2.0, dropout=0.5, name="rep").to(DEV).train().manual_seed(9)
    b.load_state_dict(a.state_dict())
    x = torch.randn(4, 32, device=DEV)
    y1, y2 = a(x), b(x)
    assert torch.equal(y1, y2)          # same name + seed -> same masks, run to run
    assert not torch.equal(a(x), y1)    # the seed advances with every training forward
