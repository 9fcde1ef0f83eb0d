"""Raw-image preprocessing on HIP: decoded RGB uint8 images -> the normalised
fp32 NCHW pixel tensor, bit-identical to the reference's torchvision transforms on PIL images:

  * mode "train": `preprocess` of src/model/dataset.py:14-19 — Resize(256) (shorter side to 256,
    the longer one int(256 * long / short)), CenterCrop(256), ToTensor, Normalize(mean 0.5,
    std ImageNet);
  * mode "retrieval": the ImageSimilarity transform of src/evidence/im2im_retrieval.py:19-27 —
    Resize((224, 224)), ToTensor, Normalize(ImageNet mean / std);
  * mode "evaluate": MisinformationPredictor's image_transform of evaluate.py:71-79 —
    Resize((256, 256)), ToTensor, Normalize(ImageNet mean / std).
`size=` overrides the (square) resize of the fixed-size modes, e.g. 224 for a ViT-B/16 predictor.

torchvision resizes PIL images with PIL's Image.resize(BILINEAR). Its taps are computed here on the
host exactly as PIL computes them (double precision, 22-bit fixed point; cached per (in, out)
size), and csrc/preprocess.hip runs PIL's integer two-pass arithmetic on the device, then ToTensor's
division and Normalize's subtract/divide in fp32. JPEG/PNG decoding stays on the host (PIL).
"""
from __future__ import annotations

import ctypes
import functools
import math

import numpy as np
import torch

from . import kernels as K

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)
MODES = {
    "train": dict(resize=256, crop=256, mean=(0.5, 0.5, 0.5), std=IMAGENET_STD),   # dataset.py:14-19
    "retrieval": dict(resize=(224, 224), crop=None, mean=IMAGENET_MEAN, std=IMAGENET_STD),  # im2im:19-27
    "evaluate": dict(resize=(256, 256), crop=None, mean=IMAGENET_MEAN, std=IMAGENET_STD),   # evaluate.py:71-79
}
_PB = 22  # PIL PRECISION_BITS (8-bit images)


class ImageDesc(ctypes.Structure):
    _fields_ = [("src", ctypes.c_void_p), ("h", ctypes.c_int64), ("w", ctypes.c_int64), ("stride", ctypes.c_int64),
                ("out_h", ctypes.c_int32), ("out_w", ctypes.c_int32), ("crop_y", ctypes.c_int32),
                ("crop_x", ctypes.c_int32), ("kx_off", ctypes.c_int64), ("ky_off", ctypes.c_int64),
                ("kx_size", ctypes.c_int32), ("ky_size", ctypes.c_int32), ("tmp_off", ctypes.c_int64)]


@functools.lru_cache(maxsize=4096)
def pil_taps(in_size: int, out_size: int):
    """PIL's precompute_coeffs + normalize_coeffs_8bpc for the bilinear filter over the whole input
    range: int32 [out_size, K + 2] records [xmin, n, k_0 .. k_{K-1}] (K = 2 ceil(support) + 1)."""
    scale = in_size / out_size
    fs = max(scale, 1.0)
    support = 1.0 * fs
    K_ = int(math.ceil(support)) * 2 + 1
    out = np.zeros((out_size, K_ + 2), np.int32)
    ss = 1.0 / fs
    for xx in range(out_size):
        center = (xx + 0.5) * scale
        xmin = max(int(center - support + 0.5), 0)
        xmax = min(int(center + support + 0.5), in_size) - xmin
        w = []
        ww = 0.0
        for x in range(xmax):
            t = abs((x + xmin - center + 0.5) * ss)
            v = 1.0 - t if t < 1.0 else 0.0
            w.append(v)
            ww += v
        out[xx, 0], out[xx, 1] = xmin, xmax
        for x, v in enumerate(w):
            v = v / ww if ww != 0.0 else v
            out[xx, 2 + x] = int(-0.5 + v * (1 << _PB)) if v < 0 else int(0.5 + v * (1 << _PB))
    return out


def resized_size(h: int, w: int, size):
    """torchvision.transforms.functional._compute_resized_output_size for PIL input: an int resizes
    the shorter side (the longer one truncated), a pair is (h, w)"""
    if isinstance(size, (tuple, list)):
        return int(size[0]), int(size[1])
    short, long_ = (w, h) if w <= h else (h, w)
    if short == size:
        return h, w
    new_short, new_long = size, int(size * long_ / short)
    return (new_long, new_short) if w <= h else (new_short, new_long)


def center_crop_origin(h: int, w: int, crop: int):
    """torchvision CenterCrop: top = int(round((h - crop) / 2.0)) (Python's round)"""
    return int(round((h - crop) / 2.0)), int(round((w - crop) / 2.0))


def _as_uint8_rgb(img):
    from PIL import Image
    if isinstance(img, Image.Image):
        return np.asarray(img.convert("RGB"), dtype=np.uint8)
    a = np.asarray(img)
    if a.dtype != np.uint8 or a.ndim != 3 or a.shape[2] != 3:
        raise ValueError("images must be PIL images or uint8 HxWx3 arrays")
    return a


class ImagePreprocessor:
    """Batch preprocessing on the GPU: __call__(list of PIL images / uint8 HWC arrays) -> fp32
    [N, 3, S, S] on `device`."""

    def __init__(self, mode="train", device="cuda", size=None):
        if mode not in MODES:
            raise ValueError(f"mode must be one of {list(MODES)}")
        self.mode, self.cfg, self.device = mode, dict(MODES[mode]), torch.device(device)
        if size is not None:
            if self.cfg["crop"]:
                raise ValueError("size= applies to the fixed-size modes (retrieval / evaluate)")
            self.cfg["resize"] = (int(size), int(size))
        c = self.cfg
        self.out_hw = (c["crop"], c["crop"]) if c["crop"] else tuple(c["resize"])
        self._mean = (ctypes.c_float * 3)(*c["mean"])
        self._std = (ctypes.c_float * 3)(*c["std"])

    def plan(self, shapes, src_ptrs):
        """Descriptors, taps and workspace for images of the given (h, w) whose uint8 HWC pixels
        sit at the device addresses src_ptrs (reusable for repeated batches of the same shapes)."""
        n = len(shapes)
        descs = (ImageDesc * n)()
        coefs, coff, toff, max_h, max_ow = [], 0, 0, 0, 0
        for i, (h, w) in enumerate(shapes):
            oh, ow = resized_size(h, w, self.cfg["resize"])
            cy, cx = center_crop_origin(oh, ow, self.cfg["crop"]) if self.cfg["crop"] else (0, 0)
            if cy < 0 or cx < 0:
                raise ValueError("image smaller than the crop after resizing")
            tx, ty = pil_taps(w, ow), pil_taps(h, oh)
            d = descs[i]
            d.src = int(src_ptrs[i])
            d.h, d.w, d.stride = h, w, 3 * w
            d.out_h, d.out_w, d.crop_y, d.crop_x = oh, ow, cy, cx
            d.kx_off, d.kx_size = coff, tx.shape[1] - 2
            coff += tx.size
            d.ky_off, d.ky_size = coff, ty.shape[1] - 2
            coff += ty.size
            d.tmp_off = toff
            toff += h * ow * 3
            coefs += [tx.reshape(-1), ty.reshape(-1)]
            max_h, max_ow = max(max_h, h), max(max_ow, ow)
        coef = torch.from_numpy(np.concatenate(coefs)).to(self.device, non_blocking=True)
        table = torch.frombuffer(bytearray(bytes(descs)), dtype=torch.uint8).to(self.device)
        ws = torch.empty(max(toff, 1), dtype=torch.uint8, device=self.device)
        return dict(n=n, table=table, coef=coef, ws=ws, max_h=max_h, max_ow=max_ow)

    def launch(self, plan, out=None):
        """Run the two preprocessing kernels for a plan -> fp32 [N, 3, S, S]"""
        Ho, Wo = self.out_hw
        if out is None:
            out = torch.empty(plan["n"], 3, Ho, Wo, device=self.device, dtype=torch.float32)
        K._check(K.lib().mmfd_resize_normalize(plan["n"], K._ptr(plan["table"]), plan["max_h"], plan["max_ow"],
                                                K._ptr(plan["coef"]), K._ptr(plan["ws"]), Ho, Wo, self._mean,
                                                self._std, K._ptr(out), K._stream()), "mmfd_resize_normalize")
        return out

    def from_device(self, src, shapes, offsets):
        """The batch whose uint8 HWC pixels already sit in the device buffer `src` (image i at byte
        offsets[i], shape shapes[i] = (h, w)) -> fp32 [N, 3, S, S]: no host staging at all
        (mmfd.hostdecode.PinnedDecodeRing uploads the decoded pixels there asynchronously)."""
        Ho, Wo = self.out_hw
        if not shapes:
            return torch.empty(0, 3, Ho, Wo, device=self.device, dtype=torch.float32)
        plan = self.plan(list(shapes), [src.data_ptr() + int(o) for o in offsets])
        out = self.launch(plan)
        out._keepalive = (src, plan)  # until the stream has consumed them
        return out

    def __call__(self, images):
        arrs = [_as_uint8_rgb(im) for im in images]
        n = len(arrs)
        Ho, Wo = self.out_hw
        if n == 0:
            return torch.empty(0, 3, Ho, Wo, device=self.device, dtype=torch.float32)
        # one host buffer and one upload for the whole batch
        sizes = [a.size for a in arrs]
        src = torch.empty(sum(sizes), dtype=torch.uint8, pin_memory=True)
        offs = np.cumsum([0] + sizes)
        for a, o in zip(arrs, offs):
            src[o:o + a.size].numpy()[:] = a.reshape(-1)
        dsrc = src.to(self.device, non_blocking=True)
        plan = self.plan([a.shape[:2] for a in arrs], [dsrc.data_ptr() + int(o) for o in offs[:-1]])
        out = self.launch(plan)
        out._keepalive = (dsrc, src, plan)  # until the stream has consumed them
        return out
