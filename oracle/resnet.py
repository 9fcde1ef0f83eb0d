"""TEST INFRASTRUCTURE ONLY (oracle).

CPU restatement of the reference's image feature extractor (im2im_retrieval.py:14-36): torchvision
resnet50 (v1.5: stride on the 3x3 conv) with the classifier removed, eval mode, output the global
average pool [N, 2048, 1, 1]. torchvision is not installed here (reference pins 0.20.1,
requirements.txt); the restatement follows torchvision's ResNet/Bottleneck definition and is
pinned against transformers' ResNetModel (same architecture, different parameter names) in
tests/golden/make_golden.py (`resnet_small.npz`). Parameters use torchvision state_dict names.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def _bn(P, n, x, eps=1e-5):
    return F.batch_norm(x, P[n + ".running_mean"], P[n + ".running_var"], P[n + ".weight"], P[n + ".bias"],
                        training=False, eps=eps)


def resnet_forward(P, x, depths=(3, 4, 6, 3)):
    x = F.relu(_bn(P, "bn1", F.conv2d(x, P["conv1.weight"], stride=2, padding=3)))
    x = F.max_pool2d(x, 3, 2, 1)
    for i, d in enumerate(depths):
        for j in range(d):
            p = f"layer{i + 1}.{j}"
            stride = 2 if (i > 0 and j == 0) else 1
            h = F.relu(_bn(P, p + ".bn1", F.conv2d(x, P[p + ".conv1.weight"])))
            h = F.relu(_bn(P, p + ".bn2", F.conv2d(h, P[p + ".conv2.weight"], stride=stride, padding=1)))
            h = _bn(P, p + ".bn3", F.conv2d(h, P[p + ".conv3.weight"]))
            if p + ".downsample.0.weight" in P:
                x = _bn(P, p + ".downsample.1", F.conv2d(x, P[p + ".downsample.0.weight"], stride=stride))
            x = F.relu(h + x)
    return F.adaptive_avg_pool2d(x, (1, 1))


def hf_to_torchvision(name):
    """transformers ResNetModel parameter name -> torchvision resnet name"""
    n = name.replace("embedder.embedder.convolution", "conv1").replace("embedder.embedder.normalization", "bn1")
    if n.startswith("encoder.stages."):
        parts = n.split(".")  # encoder.stages.S.layers.L.<rest>
        s, l, rest = int(parts[2]), int(parts[4]), parts[5:]
        pre = f"layer{s + 1}.{l}"
        if rest[0] == "shortcut":
            tail = ".".join(rest[2:])
            n = f"{pre}.downsample.{'0' if rest[1] == 'convolution' else '1'}.{tail}"
        else:  # layer.J.convolution|normalization.<tail>
            jj = int(rest[1]) + 1
            tail = ".".join(rest[3:])
            n = f"{pre}.{'conv' if rest[2] == 'convolution' else 'bn'}{jj}.{tail}"
    return n
