"""Host-side image / label transforms of the CAT-Seg data path (detectron2 v0.6
`data/transforms` semantics, which the reference reaches through its mappers and
detectron2's test `DatasetMapper`; no detectron2 / cv2 needed).

Each augmentation's `get_transform(image, sem_seg)` returns a deterministic transform with
`apply_image` / `apply_segmentation`, as in detectron2, so image and label stay aligned:

  ResizeShortestEdge        test: short edge 640, long edge <= 2560 (INPUT.MIN/MAX_SIZE_TEST,
                            the eval protocol, vizDebug/log.txt:1876); train: choice of
                            INPUT.MIN_SIZE_TRAIN (configs/config.yaml:50-51)
  RandomCropCategoryArea    RandomCrop_CategoryAreaConstraint (configs/config.yaml:54-58)
  ColorAugSSD               point_rend ColorAugSSDTransform (COLOR_AUG_SSD, config.yaml:59)
  RandomFlip                horizontal, p = 0.5

uint8 images are resized with PIL (bilinear; nearest for labels), others with torch
`F.interpolate`, as detectron2's `ResizeTransform` does.
"""
from __future__ import annotations

import random
from typing import Optional, Sequence, Tuple

import numpy as np
import torch
import torch.nn.functional as F
from PIL import Image


def resize_output_shape(h: int, w: int, short: int, max_size: int) -> Tuple[int, int]:
    """ResizeShortestEdge.get_output_shape: scale the short edge to `short`, then shrink so the
    long edge is <= max_size; round half up."""
    size = float(short)
    scale = size / min(h, w)
    newh, neww = (size, scale * w) if h < w else (scale * h, size)
    if max(newh, neww) > max_size:
        s = max_size * 1.0 / max(newh, neww)
        newh, neww = newh * s, neww * s
    return int(newh + 0.5), int(neww + 0.5)


class Transform:
    def apply_image(self, img: np.ndarray) -> np.ndarray:
        raise NotImplementedError

    def apply_segmentation(self, seg: np.ndarray) -> np.ndarray:
        return seg


class NoOp(Transform):
    def apply_image(self, img):
        return img


class ResizeTransform(Transform):
    def __init__(self, h, w, new_h, new_w, interp=Image.BILINEAR):
        self.h, self.w, self.new_h, self.new_w, self.interp = h, w, new_h, new_w, interp

    def apply_image(self, img, interp=None):
        assert img.shape[:2] == (self.h, self.w), (img.shape, self.h, self.w)
        interp = self.interp if interp is None else interp
        if img.dtype == np.uint8:
            pil = Image.fromarray(img[:, :, 0], mode="L") if img.ndim == 3 and img.shape[2] == 1 else Image.fromarray(img)
            out = np.asarray(pil.resize((self.new_w, self.new_h), interp))
            if img.ndim == 3 and img.shape[2] == 1:
                out = out[:, :, None]
            return out
        # PIL handles uint8 only: torch interpolation for the rest (labels as double, 16-bit tiff)
        t = torch.from_numpy(np.ascontiguousarray(img))
        shape = list(t.shape)
        t = t.view(shape[0], shape[1], -1).permute(2, 0, 1)[None].float()            # 1, C, H, W
        mode = {Image.NEAREST: "nearest", Image.BILINEAR: "bilinear", Image.BICUBIC: "bicubic"}[interp]
        kw = {} if mode == "nearest" else {"align_corners": False}
        t = F.interpolate(t, (self.new_h, self.new_w), mode=mode, **kw)
        shape[:2] = (self.new_h, self.new_w)
        return t[0].permute(1, 2, 0).reshape(shape).numpy().astype(img.dtype)

    def apply_segmentation(self, seg):
        return self.apply_image(seg, interp=Image.NEAREST)


class CropTransform(Transform):
    def __init__(self, x0, y0, w, h):
        self.x0, self.y0, self.w, self.h = x0, y0, w, h

    def apply_image(self, img):
        return img[self.y0:self.y0 + self.h, self.x0:self.x0 + self.w]

    apply_segmentation = apply_image


class HFlipTransform(Transform):
    def __init__(self, width):
        self.width = width

    def apply_image(self, img):
        return np.ascontiguousarray(img[:, ::-1])

    apply_segmentation = apply_image


class ResizeShortestEdge:
    def __init__(self, short_edge_length, max_size=2 ** 31 - 1, sample_style="range", interp=Image.BILINEAR):
        if isinstance(short_edge_length, int):
            short_edge_length = (short_edge_length, short_edge_length)
        self.short = tuple(short_edge_length)
        self.max_size, self.interp = max_size, interp
        self.is_range = sample_style == "range"

    def get_transform(self, image, sem_seg=None):
        h, w = image.shape[:2]
        size = (np.random.randint(self.short[0], self.short[1] + 1) if self.is_range
                else int(np.random.choice(self.short)))
        if size == 0:
            return NoOp()
        nh, nw = resize_output_shape(h, w, size, self.max_size)
        return ResizeTransform(h, w, nh, nw, self.interp)

    def __repr__(self):
        return f"ResizeShortestEdge(short_edge_length={self.short}, max_size={self.max_size})"


class RandomCropCategoryArea:
    """RandomCrop_CategoryAreaConstraint: up to 10 draws of a crop in which no single category
    (ignore label excluded) covers more than `single_category_max_area` of the pixels."""

    def __init__(self, crop_type: str, crop_size: Sequence[float], single_category_max_area: float = 1.0,
                 ignored_category: Optional[int] = None):
        self.crop_type, self.crop_size = crop_type, tuple(crop_size)
        self.max_area, self.ignored = single_category_max_area, ignored_category

    def crop_size_for(self, h, w):
        ch, cw = self.crop_size
        if self.crop_type == "relative":
            return int(h * ch + 0.5), int(w * cw + 0.5)
        if self.crop_type == "relative_range":
            rh, rw = np.asarray(self.crop_size, dtype=np.float32)
            rh, rw = rh + np.random.rand() * (1 - rh), rw + np.random.rand() * (1 - rw)
            return int(h * rh + 0.5), int(w * rw + 0.5)
        if self.crop_type == "absolute":
            return min(int(ch), h), min(int(cw), w)
        if self.crop_type == "absolute_range":
            lo, hi = self.crop_size
            return np.random.randint(min(h, lo), min(h, hi) + 1), np.random.randint(min(w, lo), min(w, hi) + 1)
        raise NotImplementedError(f"Unknown crop type {self.crop_type}")

    def get_transform(self, image, sem_seg=None):
        h, w = image.shape[:2]
        if self.max_area >= 1.0 or sem_seg is None:
            ch, cw = self.crop_size_for(h, w)
            # detectron2 RandomCrop.get_transform draws h0 first, then w0
            y0 = np.random.randint(h - ch + 1)
            x0 = np.random.randint(w - cw + 1)
            return CropTransform(x0, y0, cw, ch)
        for _ in range(10):
            ch, cw = self.crop_size_for(h, w)
            y0, x0 = np.random.randint(h - ch + 1), np.random.randint(w - cw + 1)
            labels, cnt = np.unique(sem_seg[y0:y0 + ch, x0:x0 + cw], return_counts=True)
            if self.ignored is not None:
                cnt = cnt[labels != self.ignored]
            if len(cnt) > 1 and np.max(cnt) < np.sum(cnt) * self.max_area:
                break
        return CropTransform(x0, y0, cw, ch)


def _rgb_to_hsv_u8(img):
    """OpenCV's uint8 HSV convention (H in [0, 180), S and V in [0, 255])."""
    f = img.astype(np.float32)
    r, g, b = f[..., 0], f[..., 1], f[..., 2]
    v = f.max(-1)
    mn = f.min(-1)
    d = v - mn
    s = np.where(v > 0, 255.0 * d / np.maximum(v, 1e-6), 0.0)
    dd = np.maximum(d, 1e-6)
    h = np.where(v == r, 60.0 * (g - b) / dd, np.where(v == g, 120.0 + 60.0 * (b - r) / dd, 240.0 + 60.0 * (r - g) / dd))
    h = np.where(d == 0, 0.0, h) % 360.0
    return np.stack([np.round(h / 2) % 180, np.round(s), v], -1).astype(np.uint8)


def _hsv_to_rgb_u8(hsv):
    h = hsv[..., 0].astype(np.float32) * 2.0
    s = hsv[..., 1].astype(np.float32) / 255.0
    v = hsv[..., 2].astype(np.float32)
    c = v * s
    x = c * (1 - np.abs((h / 60.0) % 2 - 1))
    m = v - c
    z = np.zeros_like(c)
    k = (h // 60).astype(np.int32) % 6
    rgb = np.select([k[..., None] == i for i in range(6)],
                    [np.stack(t, -1) for t in ((c, x, z), (x, c, z), (z, c, x), (z, x, c), (x, z, c), (c, z, x))])
    return np.clip(np.round(rgb + m[..., None]), 0, 255).astype(np.uint8)


class ColorAugSSD(Transform):
    """point_rend ColorAugSSDTransform: random brightness (+-32), then contrast [0.5, 1.5] and
    saturation [0.5, 1.5] / hue (+-18 on the 180-step wheel) in one of two orders.  The
    reference implementation uses cv2's HSV conversion (cv2 is absent here; same uint8
    convention, restated in numpy)."""

    def __init__(self, brightness_delta=32, contrast_low=0.5, contrast_high=1.5, saturation_low=0.5,
                 saturation_high=1.5, hue_delta=18):
        self.bd, self.cl, self.ch = brightness_delta, contrast_low, contrast_high
        self.sl, self.sh, self.hd = saturation_low, saturation_high, hue_delta

    def get_transform(self, image, sem_seg=None):
        return self

    @staticmethod
    def _convert(img, alpha=1.0, beta=0.0):
        return np.clip(img.astype(np.float32) * alpha + beta, 0, 255).astype(np.uint8)

    def apply_image(self, img):
        if random.randrange(2):
            img = self._convert(img, beta=random.uniform(-self.bd, self.bd))
        order = (self._contrast, self._saturation, self._hue) if random.randrange(2) else \
            (self._saturation, self._hue, self._contrast)
        for f in order:
            img = f(img)
        return img

    def _contrast(self, img):
        return self._convert(img, alpha=random.uniform(self.cl, self.ch)) if random.randrange(2) else img

    def _saturation(self, img):
        if random.randrange(2):
            hsv = _rgb_to_hsv_u8(img)
            hsv[..., 1] = self._convert(hsv[..., 1], alpha=random.uniform(self.sl, self.sh))
            return _hsv_to_rgb_u8(hsv)
        return img

    def _hue(self, img):
        if random.randrange(2):
            hsv = _rgb_to_hsv_u8(img)
            hsv[..., 0] = (hsv[..., 0].astype(np.int32) + random.randint(-self.hd, self.hd)) % 180
            return _hsv_to_rgb_u8(hsv)
        return img


class RandomFlip:
    def __init__(self, prob=0.5):
        self.prob = prob

    def get_transform(self, image, sem_seg=None):
        return HFlipTransform(image.shape[1]) if np.random.rand() < self.prob else NoOp()


def apply_augmentations(augs, image, sem_seg=None):
    """Apply each augmentation's transform in turn to the image (and label map)."""
    tfms = []
    for aug in augs:
        t = aug.get_transform(image, sem_seg)
        image = t.apply_image(image)
        if sem_seg is not None:
            sem_seg = t.apply_segmentation(sem_seg)
        tfms.append(t)
    return image, sem_seg, tfms
