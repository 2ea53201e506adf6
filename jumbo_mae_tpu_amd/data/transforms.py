"""Image transforms (PIL / numpy; torchvision and timm are not installed).

Reference ``create_transforms`` (/root/reference/src/dataset.py:56-82):
  train: RandomResizedCrop(size, scale=(0.2, 1), bicubic) | "src": Resize+RandomCrop(pad 4,
         reflect) | "none": Resize+CenterCrop; HorizontalFlip; RandAugment/AugMix/AutoAugment or
         identity; ColorJitter(b, c, s); RandomErasing(p, value="random"); PILToTensor (uint8 CHW)
  valid: Resize(int(size / crop_ratio), bicubic) -> CenterCrop(size) -> PILToTensor
Semantics follow torchvision (RRC: 10 attempts of (scale, log-ratio) sampling, then a central
fallback crop clamped to the ratio range).
"""

from __future__ import annotations

import math
import random

import numpy as np
from PIL import Image, ImageEnhance

BICUBIC = Image.BICUBIC


class Compose:
    def __init__(self, ts):
        self.ts = [t for t in ts if t is not None]

    def __call__(self, x):
        for t in self.ts:
            x = t(x)
        return x


class RandomResizedCrop:
    def __init__(self, size, scale=(0.08, 1.0), ratio=(3 / 4, 4 / 3), interpolation=BICUBIC):
        self.size = (size, size) if isinstance(size, int) else tuple(size)
        self.scale, self.ratio, self.interpolation = scale, ratio, interpolation

    def get_params(self, w, h):
        area = w * h
        log_ratio = (math.log(self.ratio[0]), math.log(self.ratio[1]))
        for _ in range(10):
            target_area = area * random.uniform(*self.scale)
            aspect = math.exp(random.uniform(*log_ratio))
            cw = int(round(math.sqrt(target_area * aspect)))
            ch = int(round(math.sqrt(target_area / aspect)))
            if 0 < cw <= w and 0 < ch <= h:
                return random.randint(0, h - ch), random.randint(0, w - cw), ch, cw
        in_ratio = w / h
        if in_ratio < min(self.ratio):
            cw = w
            ch = int(round(cw / min(self.ratio)))
        elif in_ratio > max(self.ratio):
            ch = h
            cw = int(round(ch * max(self.ratio)))
        else:
            cw, ch = w, h
        return (h - ch) // 2, (w - cw) // 2, ch, cw

    def __call__(self, img):
        i, j, h, w = self.get_params(*img.size)
        return img.resize(self.size[::-1], self.interpolation, box=(j, i, j + w, i + h))


class Resize:
    """Resize the shorter side to ``size`` (torchvision int-size semantics)."""

    def __init__(self, size, interpolation=BICUBIC):
        self.size, self.interpolation = size, interpolation

    def __call__(self, img):
        w, h = img.size
        if w <= h:
            nw, nh = self.size, int(self.size * h / w)
        else:
            nh, nw = self.size, int(self.size * w / h)
        if (nw, nh) == (w, h):
            return img
        return img.resize((nw, nh), self.interpolation)


class CenterCrop:
    def __init__(self, size):
        self.size = size

    def __call__(self, img):
        w, h = img.size
        th = tw = self.size
        i = int(round((h - th) / 2.0))
        j = int(round((w - tw) / 2.0))
        return img.crop((j, i, j + tw, i + th))


class RandomCrop:
    def __init__(self, size, padding=0, padding_mode="reflect"):
        self.size, self.padding, self.mode = size, padding, padding_mode

    def __call__(self, img):
        a = np.asarray(img)
        if self.padding:
            p = self.padding
            a = np.pad(a, ((p, p), (p, p), (0, 0)), mode="reflect" if self.mode == "reflect" else "constant")
        h, w = a.shape[:2]
        i = random.randint(0, h - self.size)
        j = random.randint(0, w - self.size)
        return Image.fromarray(np.ascontiguousarray(a[i:i + self.size, j:j + self.size]))


class RandomHorizontalFlip:
    def __init__(self, p=0.5):
        self.p = p

    def __call__(self, img):
        return img.transpose(Image.FLIP_LEFT_RIGHT) if random.random() < self.p else img


class ColorJitter:
    """Brightness / contrast / saturation jitter with factors in [1-x, 1+x], random order."""

    def __init__(self, brightness=0.0, contrast=0.0, saturation=0.0):
        self.ops = []
        for name, v in (("b", brightness), ("c", contrast), ("s", saturation)):
            if v > 0:
                self.ops.append((name, max(0.0, 1 - v), 1 + v))

    def __call__(self, img):
        ops = list(self.ops)
        random.shuffle(ops)
        for name, lo, hi in ops:
            f = random.uniform(lo, hi)
            if name == "b":
                img = ImageEnhance.Brightness(img).enhance(f)
            elif name == "c":
                img = ImageEnhance.Contrast(img).enhance(f)
            else:
                img = ImageEnhance.Color(img).enhance(f)
        return img


class PILToArray:
    """PIL -> uint8 CHW numpy array (PILToTensor)."""

    def __call__(self, img):
        return np.ascontiguousarray(np.asarray(img.convert("RGB"), dtype=np.uint8).transpose(2, 0, 1))


def erase_fill(noise: np.ndarray) -> np.ndarray:
    """float noise -> uint8 the way ``uint8_tensor[...] = float_tensor`` stores it (truncate, wrap)."""
    return (np.trunc(noise).astype(np.int64) & 255).astype(np.uint8)


class RandomErasing:
    """torchvision v2 RandomErasing(p, scale=(0.02, 0.33), ratio=(0.3, 3.3), value="random") on a
    uint8 CHW array (/root/reference/src/dataset.py:74).

    ``value="random"`` in torchvision v2 draws the patch as float32 standard-normal noise and
    assigns it into the uint8 image, i.e. each value is truncated toward zero and wrapped modulo
    256 (-1.3 -> 255, 0.9 -> 0, 2.2 -> 2): the erased patch is near-black with a sprinkle of
    near-white pixels.  That effective fill is reproduced here (``erase_fill``).  torchvision is
    not installed in this image, so the match is pinned to torch's own float->uint8 assignment in
    tests/test_data.py, not to torchvision itself (parity unpinned at the library level)."""

    def __init__(self, p=0.5, scale=(0.02, 0.33), ratio=(0.3, 3.3)):
        self.p, self.scale, self.ratio = p, scale, ratio

    def __call__(self, a):
        if random.random() >= self.p:
            return a
        c, h, w = a.shape
        area = h * w
        log_ratio = (math.log(self.ratio[0]), math.log(self.ratio[1]))
        for _ in range(10):
            ea = area * random.uniform(*self.scale)
            ar = math.exp(random.uniform(*log_ratio))
            eh = int(round(math.sqrt(ea * ar)))
            ew = int(round(math.sqrt(ea / ar)))
            if eh < h and ew < w:
                i = random.randint(0, h - eh)
                j = random.randint(0, w - ew)
                a = a.copy()
                a[:, i:i + eh, j:j + ew] = erase_fill(np.random.standard_normal((c, eh, ew)).astype(np.float32))
                return a
        return a


def auto_augment_factory(name: str, image_size: int):
    from .autoaugment import augmix_transform, auto_augment_transform, rand_augment_transform
    from .constants import IMAGENET_DEFAULT_MEAN

    hparams = {"translate_const": int(image_size * 0.45),
               "img_mean": tuple(int(m * 255) for m in IMAGENET_DEFAULT_MEAN)}
    if name == "none":
        return None
    if name.startswith("rand"):
        return rand_augment_transform(name, hparams)
    if name.startswith("augmix"):
        hparams["translate_pct"] = 0.3
        return augmix_transform(name, hparams)
    return auto_augment_transform(name, hparams)


def create_transforms(random_crop="rrc", image_size=224, auto_augment="none", color_jitter=0.0,
                      random_erasing=0.0, test_crop_ratio=0.875):
    if random_crop == "rrc":
        train = [RandomResizedCrop(image_size, scale=(0.2, 1.0), interpolation=BICUBIC)]
    elif random_crop == "src":
        train = [Resize(image_size), RandomCrop(image_size, padding=4, padding_mode="reflect")]
    elif random_crop == "none":
        train = [Resize(image_size), CenterCrop(image_size)]
    else:
        raise ValueError(random_crop)
    train += [
        RandomHorizontalFlip(),
        auto_augment_factory(auto_augment, image_size),
        ColorJitter(color_jitter, color_jitter, color_jitter) if color_jitter > 0 else None,
        PILToArray(),
        RandomErasing(random_erasing) if random_erasing > 0 else None,
    ]
    valid = [Resize(int(image_size / test_crop_ratio)), CenterCrop(image_size), PILToArray()]
    return Compose(train), Compose(valid)
