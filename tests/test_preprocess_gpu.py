"""Raw-image preprocessing on HIP (csrc/preprocess.hip, mmfd.preprocess.ImagePreprocessor) against
the CPU oracle (oracle/preprocess.py: PIL's own resize + torchvision's crop / ToTensor / Normalize
rules). The bar is bit-exact fp32 output: the uint8 resample is PIL's integer arithmetic and the
normalisation is the same IEEE fp32 ops."""
import numpy as np
import pytest
import torch
from PIL import Image

import mmfd  # noqa: F401
from mmfd.preprocess import MODES, ImagePreprocessor
from oracle.preprocess import preprocess

pytestmark = pytest.mark.gpu

SIZES = [(375, 500), (500, 375), (256, 256), (256, 300), (300, 256), (100, 90), (31, 7), (1024, 683), (224, 224),
         (257, 1000)]


@pytest.mark.parametrize("mode", ["train", "retrieval", "evaluate"])
def test_batch_bit_exact_vs_pil_torchvision(mode):
    rng = np.random.default_rng(7)
    imgs = [Image.fromarray(rng.integers(0, 256, (h, w, 3), dtype=np.uint8)) for h, w in SIZES]
    imgs.append(imgs[0].convert("L"))     # grayscale -> RGB conversion on the host
    imgs.append(imgs[1].convert("RGBA"))
    out = ImagePreprocessor(mode)(imgs).cpu().numpy()
    c = MODES[mode]
    for i, im in enumerate(imgs):
        ref = preprocess(im, c["resize"], c["crop"], c["mean"], c["std"])
        assert out[i].shape == ref.shape
        assert np.array_equal(out[i], ref), (mode, i, np.abs(out[i] - ref).max())


def test_empty_and_errors():
    pre = ImagePreprocessor("train")
    assert pre([]).shape == (0, 3, 256, 256)
    with pytest.raises(ValueError):
        pre([np.zeros((10, 10), np.uint8)])
    with pytest.raises(ValueError):
        ImagePreprocessor("nope")


def test_size_override_matches_square_resize():
    """MisinformationPredictor with a 224 ViT: Resize((224, 224)) + ImageNet normalisation."""
    rng = np.random.default_rng(9)
    imgs = [Image.fromarray(rng.integers(0, 256, (h, w, 3), dtype=np.uint8)) for h, w in SIZES[:4]]
    out = ImagePreprocessor("evaluate", size=224)(imgs).cpu().numpy()
    c = MODES["evaluate"]
    for i, im in enumerate(imgs):
        assert np.array_equal(out[i], preprocess(im, (224, 224), None, c["mean"], c["std"]))
