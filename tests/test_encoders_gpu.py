"""BERT / ViT encoders on the HIP path vs transformers' own outputs (fixtures) and the CPU oracle.
fp32 tolerances: hidden states 1e-4 abs, parameter gradients 5e-4 relative to the tensor max."""
import json
import os

import numpy as np
import pytest
import torch

import mmfd
from mmfd.encoders import BertConfig, BertModel, ViTConfig, ViTModel
from oracle import encoders as OE
from oracle.dropout_hash import make_drop
from oracle.fusion_head import init_params_like_reference

pytestmark = pytest.mark.gpu
DEV = "cuda"
G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _z(name):
    return np.load(os.path.join(G, name), allow_pickle=False)


def _close(got, ref, tol):
    got = torch.as_tensor(got).detach().double().cpu()
    ref = torch.as_tensor(ref).detach().double().cpu() if torch.is_tensor(ref) else torch.from_numpy(np.asarray(ref)).double()
    assert got.shape == ref.shape, (got.shape, ref.shape)
    err = (got - ref).abs().max().item()
    assert err <= tol, f"{err:.3e} > {tol:.1e}"


def _load(m, z):
    sd = {k[6:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("param/")}
    m.load_state_dict(sd)
    return m.to(DEV)


def test_bert_small_matches_transformers():
    z = _z("bert_small.npz")
    c = json.loads(str(z["config"]))
    m = _load(BertModel(BertConfig(**c)), z).eval()
    out = m(input_ids=torch.from_numpy(z["input_ids"]).to(DEV), attention_mask=torch.from_numpy(z["attention_mask"]).to(DEV),
            token_type_ids=torch.from_numpy(z["token_type_ids"]).to(DEV)).last_hidden_state
    _close(out, z["out"], 1e-4)
    (out * torch.from_numpy(z["R"]).to(DEV)).sum().backward()
    for n, p in m.named_parameters():
        ref = z["grad/" + n]
        _close(p.grad, ref, 5e-4 * max(1.0, np.abs(ref).max()))


def test_vit_small_matches_transformers():
    z = _z("vit_small.npz")
    c = json.loads(str(z["config"]))
    m = _load(ViTModel(ViTConfig(**c)), z).eval()
    out = m(torch.from_numpy(z["pixel_values"]).to(DEV)).last_hidden_state
    _close(out, z["out"], 1e-4)
    (out * torch.from_numpy(z["R"]).to(DEV)).sum().backward()
    for n, p in m.named_parameters():
        ref = z["grad/" + n]
        _close(p.grad, ref, 5e-4 * max(1.0, np.abs(ref).max()))


def test_bert_train_mode_dropout_matches_oracle():
    z = _z("bert_small.npz")
    c = json.loads(str(z["config"]))
    m = _load(BertModel(BertConfig(**c)), z).train()
    m.manual_seed(99)
    P = {k[6:]: torch.from_numpy(z[k]).clone().requires_grad_(True) for k in z.files if k.startswith("param/")}
    ids, mask, tts = (torch.from_numpy(z[k]) for k in ("input_ids", "attention_mask", "token_type_ids"))
    out = m(input_ids=ids.to(DEV), attention_mask=mask.to(DEV), token_type_ids=tts.to(DEV)).last_hidden_state
    ref = OE.bert_forward(P, ids, mask, tts, num_layers=c["num_hidden_layers"], num_heads=c["num_attention_heads"],
                          drop=make_drop(99, 0.1))
    _close(out, ref, 1e-4)
    R = torch.from_numpy(z["R"])
    (out * R.to(DEV)).sum().backward()
    (ref * R).sum().backward()
    for n, p in m.named_parameters():
        _close(p.grad, P[n].grad, 5e-4 * max(1.0, P[n].grad.abs().max().item()))


@pytest.mark.parametrize("precision,tol", [("fp32", 2e-4), ("bf16", 0.25)])
def test_bert_base_full_size(precision, tol):
    z = _z("bert_base.npz")
    m = BertModel(BertConfig())
    m.load_state_dict(init_params_like_reference(json.loads(str(z["param_names"])), int(z["seed"])))
    m = m.to(DEV).eval().set_precision(precision)
    with torch.no_grad():
        out = m(input_ids=torch.from_numpy(z["input_ids"]).to(DEV),
                attention_mask=torch.from_numpy(z["attention_mask"]).to(DEV)).last_hidden_state
    _close(out.float(), z["out"], tol)


@pytest.mark.parametrize("precision,tol", [("fp32", 2e-4), ("bf16", 0.25)])
def test_vit_base_full_size(precision, tol):
    z = _z("vit_base.npz")
    m = ViTModel(ViTConfig())
    m.load_state_dict(init_params_like_reference(json.loads(str(z["param_names"])), int(z["seed"])))
    m = m.to(DEV).eval().set_precision(precision)
    with torch.no_grad():
        out = m(torch.from_numpy(z["pixel_values"]).float().to(DEV)).last_hidden_state
    _close(out.float(), z["out"], tol)
