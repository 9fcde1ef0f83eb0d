"""CPU oracle for raw-image preprocessing (TEST INFRASTRUCTURE ONLY: imported by tests/ and
bench.py's cpu_baseline, never by the product path).

Restates torchvision's transforms as the reference composes them — Resize(256) + CenterCrop(256)
+ ToTensor + Normalize(mean 0.5, ImageNet std) at src/model/dataset.py:14-19, and
Resize((224, 224)) + ToTensor + Normalize(ImageNet) at src/evidence/im2im_retrieval.py:19-27, and
Resize((256, 256)) + ToTensor + Normalize(ImageNet) at evaluate.py:71-79 —
on top of PIL itself: torchvision (pinned 0.20.1, absent here) resizes PIL images with
Image.resize(BILINEAR), crops with Image.crop, converts with np.asarray / 255 in fp32 and
normalises with fp32 sub / div, so PIL (importable here and on the GPU box) is the reference's
own resampling code. The size / crop-origin rules of torchvision are restated (cited below).
"""
import numpy as np


def resized_size(h, w, size):
    """torchvision/transforms/functional.py _compute_resized_output_size (PIL path, max_size None)"""
    if isinstance(size, (tuple, list)):
        return int(size[0]), int(size[1])
    short, long_ = (w, h) if w <= h else (h, w)
    if short == size:
        return h, w
    new_short, new_long = size, int(size * long_ / short)
    return (new_long, new_short) if w <= h else (new_short, new_long)


def preprocess(img, resize, crop, mean, std):
    """PIL image -> fp32 [3, S, S] exactly as the reference's transform composes it"""
    from PIL import Image
    img = img.convert("RGB")
    w, h = img.size
    oh, ow = resized_size(h, w, resize)
    if (oh, ow) != (h, w):
        img = img.resize((ow, oh), Image.BILINEAR)
    if crop is not None:
        top, left = int(round((oh - crop) / 2.0)), int(round((ow - crop) / 2.0))
        img = img.crop((left, top, left + crop, top + crop))
    a = np.asarray(img, dtype=np.uint8).transpose(2, 0, 1).astype(np.float32) / np.float32(255)
    m = np.asarray(mean, np.float32)[:, None, None]
    s = np.asarray(std, np.float32)[:, None, None]
    return (a - m) / s
