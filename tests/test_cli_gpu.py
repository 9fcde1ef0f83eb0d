"""The reference's training entry point (train.py:24-85, 311-434) on the HIP path, in its default
--pre_embed mode (train.py:127-132): the per-sample embedding store (preprocess_embeddings.py:95-114
layout, here the npz-directory form mmfd.preembed writes when h5py is absent) read by
MisinformationDataset(pre_embed=True), the 4-path head trained by mmfd.train.main, checkpoints in
the reference's layout (checkpoint-{epoch}-{step}/model.pt every --save_every, train.py:234-242).

1 step: the saved model_state_dict equals the reference's own `train_epoch` step
(tests/golden/fusion_small.npz, produced by tests/golden/make_golden.py from the reference) within
the tolerance of tests/test_fusion_gpu.py::test_train_step_matches_reference_train_epoch.
2 steps (two epochs of the one full batch): equal to the oracle's two steps (oracle/fusion_head.py
+ torch.optim.AdamW) within 2 lr on elements whose gradient is fp32 noise and 1e-5 elsewhere.
"""
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
ARCH = ["--text_input_dim", "48", "--image_input_dim", "40", "--embed_dim", "32", "--num_heads", "4",
        "--hidden_dim", "16", "--dropout", "0"]


def _store(tmp_path, z):
    d = tmp_path / "train_embeddings"
    os.makedirs(d)
    for i in range(z["X_t"].shape[0]):
        np.savez(d / f"{i}.npz", claim_text_embeds=z["X_t"][i], doc_text_embeds=z["E_t"][i],
                 claim_image_embeds=z["X_i"][i], doc_image_embeds=z["E_i"][i], labels=z["labels"][i])
    init = {k[len("init/"):]: torch.from_numpy(z[k]) for k in z.files if k.startswith("init/")}
    torch.save({"model_state_dict": init}, tmp_path / "init.pt")
    return str(tmp_path / "train.csv"), str(tmp_path / "init.pt")


def _run(tmp_path, extra):
    from mmfd.train import main, parse_args
    z = np.load(os.path.join(G, "fusion_small.npz"))
    csv, init = _store(tmp_path, z)
    out = str(tmp_path / "out")
    args = parse_args(["--pre_embed", "--train_data", csv, "--batch_size", "2", "--num_workers", "0",
                       "--init_checkpoint", init, "--output_dir", out, "--save_every", "1", "--log_every", "1",
                       "--precision", "fp32", *ARCH, *extra])
    tr, steps = main(args)
    return z, out, tr, steps


def test_cli_pre_embed_one_step_matches_reference_train_epoch(tmp_path):
    z, out, tr, steps = _run(tmp_path, ["--epochs", "1", "--steps", "1"])
    assert steps == 1
    ck = torch.load(os.path.join(out, "checkpoint-0-0", "model.pt"), map_location="cpu", weights_only=True)
    assert set(ck) == {"global_step", "epoch", "model_state_dict", "optimizer_state_dict"}
    assert ck["global_step"] == 0 and ck["epoch"] == 0
    for k, v in ck["model_state_dict"].items():
        ref = torch.from_numpy(z["post/" + k]).double()
        diff = (v.double() - ref).abs()
        assert diff.max().item() <= 2.0001e-4 + 1e-6, k
        if "grad/" + k in z.files:
            solid = torch.from_numpy(z["grad/" + k]).abs() > 1e-6
            assert (diff[solid].max().item() if solid.any() else 0.0) <= 2e-6, k
    rec = [json.loads(line) for line in open(os.path.join(out, "metrics.jsonl"))]
    assert abs(rec[0]["train/total_loss"] - float(z["train_total_loss"])) < 1e-4
    for p in ("text_text", "text_image", "image_text", "image_image"):
        assert abs(rec[0][f"train/{p}_loss"] - float(z[f"train_loss_{p}"])) < 1e-4
        assert f"train/{p}_accuracy" in rec[0] and f"train/{p}_f1" in rec[0]


def test_cli_pre_embed_two_steps_match_oracle(tmp_path):
    from oracle import fusion_head as OF
    z, out, tr, steps = _run(tmp_path, ["--epochs", "2", "--steps", "2"])
    assert steps == 2 and os.path.exists(os.path.join(out, "checkpoint-1-1", "model.pt"))
    P = {k[len("init/"):]: torch.from_numpy(z[k]).clone().requires_grad_(True) for k in z.files if k.startswith("init/")}
    opt = torch.optim.AdamW(list(P.values()), lr=1e-4)
    X = [torch.from_numpy(z[k]) for k in ("X_t", "X_i", "E_t", "E_i")]
    noisy = {}
    for _ in range(2):
        opt.zero_grad(set_to_none=True)
        tot, _ = OF.path_loss(OF.model_forward(P, *X, num_heads=4), torch.from_numpy(z["labels"]))
        tot.backward()
        for k, p in P.items():
            if p.grad is not None:
                noisy[k] = noisy.get(k, torch.zeros_like(p, dtype=torch.bool)) | (p.grad.abs() < 1e-6)
        opt.step()
    ck = torch.load(os.path.join(out, "checkpoint-1-1", "model.pt"), map_location="cpu", weights_only=True)
    for k, v in ck["model_state_dict"].items():
        diff = (v.double() - P[k].detach().double()).abs()
        assert diff.max().item() <= 4.0002e-4 + 1e-6, k
        if k in noisy:
            solid = ~noisy[k]
            assert (diff[solid].max().item() if solid.any() else 0.0) <= 1e-5, k
