"""DeBERTa-v3 text encoder (the reference's default, train.py:330-331) on the HIP path vs the
transformers fixture (tests/golden/deberta_small.npz, L=300: the long-sequence attention path,
one padded row) and vs the CPU oracle (oracle/deberta.py) at the deberta-v3-xsmall shape.
Tolerances: fp32 1e-4 abs vs the fixture, 1e-3 abs at the xsmall shape (north_star's logit bar);
bf16 0.25 max abs on the 12-layer LayerNorm'd outputs (the bar of the BERT / ViT full-size bf16
tests, test_encoders_gpu.py) plus 1e-2 mean abs, which a wrong index or mask would exceed."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _small_cfg(**kw):
    from mmfd.deberta import DebertaV2Config
    c = dict(vocab_size=1000, hidden_size=64, num_hidden_layers=2, num_attention_heads=2, intermediate_size=128)
    c.update(kw)
    return DebertaV2Config(**c)


def test_deberta_matches_transformers_fixture():
    from mmfd.deberta import DebertaV2Model
    z = np.load(os.path.join(G, "deberta_small.npz"))
    m = DebertaV2Model(_small_cfg())
    m.load_state_dict({k[2:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("w.")})
    m = m.cuda().eval()
    with torch.no_grad():
        out = m(input_ids=torch.from_numpy(z["input_ids"]).cuda(),
                attention_mask=torch.from_numpy(z["attention_mask"]).cuda()).last_hidden_state
    torch.cuda.synchronize()
    err = (out.cpu() - torch.from_numpy(z["last_hidden_state"])).abs().max().item()
    assert err < 1e-4, err


def _oracle(m, ids, mask):
    from oracle.deberta import deberta_forward
    P = {k: v.detach().float().cpu() for k, v in m.state_dict().items()}
    with torch.no_grad():
        return deberta_forward(P, ids, mask, num_layers=m.config.num_hidden_layers,
                               num_heads=m.config.num_attention_heads, eps=m.config.layer_norm_eps)


@pytest.mark.parametrize("precision,L,tol", [("fp32", 128, 1e-3), ("bf16", 128, 0.25), ("bf16", 200, 0.25),
                                             ("fp32", 512, 1e-3), ("bf16", 512, 0.25)])
def test_deberta_xsmall_vs_oracle(precision, L, tol):
    """deberta-v3-xsmall shape (hidden 384, 6 heads, 12 layers, 256 buckets) with random init;
    ragged masks (one row padded to half length); L <= 256 runs the resident-K/V attention kernels
    with the batch-strided bias (fp32 and bf16), L = 512 the streaming ones (the shape the
    pre-embedding bench times in bf16)"""
    from mmfd.deberta import DebertaV2Model
    torch.manual_seed(3)
    m = DebertaV2Model().cuda().eval().set_precision(precision)
    g = torch.Generator().manual_seed(L)
    B = 2
    ids = torch.randint(1, 128100, (B, L), generator=g)
    mask = torch.ones(B, L, dtype=torch.long)
    mask[1, L // 2:] = 0
    ids[1, L // 2:] = 0
    with torch.no_grad():
        out = m(input_ids=ids.cuda(), attention_mask=mask.cuda()).last_hidden_state
    torch.cuda.synchronize()
    ref = _oracle(m, ids, mask)
    diff = (out.float().cpu() - ref).abs()
    assert diff.max().item() < tol, (precision, L, diff.max().item())
    assert diff.mean().item() < (1e-2 if precision == "bf16" else 1e-4), (precision, L, diff.mean().item())


def test_deberta_is_inference_only():
    from mmfd.deberta import DebertaV2Model
    m = DebertaV2Model(_small_cfg()).cuda()
    ids = torch.ones(1, 8, dtype=torch.long, device="cuda")
    with pytest.raises(NotImplementedError):
        m(input_ids=ids)
    with torch.no_grad():
        assert m(input_ids=ids).last_hidden_state.shape == (1, 8, 64)
