"""RandAugment / AugMix / AutoAugment with timm's config-string grammar (timm not installed).

Reference: ``auto_augment_factory`` (/root/reference/src/dataset.py:41-53) calls timm's
``rand_augment_transform`` / ``augment_and_mix_transform`` / ``auto_augment_transform`` with
hparams {translate_const: 0.45*size, img_mean}.  Grammar: ``rand-m9-mstd0.5-inc1`` (n ops per
image, magnitude m of 10, Gaussian magnitude noise mstd, the "increasing" op set for inc1,
per-op probability p=0.5), ``augmix-m3-w3-d-1`` (width, depth, alpha, blended), ``original`` /
``v0`` AutoAugment ImageNet policies.  Level -> argument mappings follow timm's definitions.
"""

from __future__ import annotations

import random

import numpy as np
from PIL import Image, ImageEnhance, ImageOps

_MAX = 10.0
_FILL = (124, 116, 104)
_RESAMPLE = (Image.BILINEAR, Image.BICUBIC)


def _neg(v):
    return -v if random.random() > 0.5 else v


def _affine(img, matrix, hp):
    return img.transform(img.size, Image.AFFINE, matrix, resample=random.choice(_RESAMPLE),
                         fillcolor=hp.get("img_mean", _FILL))


# ---- ops: (img, level, hparams) -> img
def auto_contrast(img, lvl, hp):
    return ImageOps.autocontrast(img)


def equalize(img, lvl, hp):
    return ImageOps.equalize(img)


def invert(img, lvl, hp):
    return ImageOps.invert(img)


def rotate(img, lvl, hp):
    deg = _neg(lvl / _MAX * 30.0)
    return img.rotate(deg, resample=random.choice(_RESAMPLE), fillcolor=hp.get("img_mean", _FILL))


def _posterize_bits(img, bits):
    bits = int(bits)
    if bits >= 8:
        return img
    return ImageOps.posterize(img, max(bits, 0))


def posterize(img, lvl, hp):  # timm "Posterize": int(level/10*4)
    return _posterize_bits(img, int(lvl / _MAX * 4))


def posterize_increasing(img, lvl, hp):
    return _posterize_bits(img, 4 - int(lvl / _MAX * 4))


def posterize_original(img, lvl, hp):
    return _posterize_bits(img, int(lvl / _MAX * 4) + 4)


def solarize(img, lvl, hp):
    return ImageOps.solarize(img, int(lvl / _MAX * 256))


def solarize_increasing(img, lvl, hp):
    return ImageOps.solarize(img, 256 - int(lvl / _MAX * 256))


def solarize_add(img, lvl, hp, thresh=128):
    add = int(lvl / _MAX * 110)
    a = np.asarray(img).astype(np.int32)
    a = np.where(a < thresh, np.minimum(a + add, 255), a)
    return Image.fromarray(a.astype(np.uint8))


def _enhance(cls, factor):
    return lambda img: cls(img).enhance(factor)


def _enh_level(lvl):
    return lvl / _MAX * 1.8 + 0.1


def _enh_inc_level(lvl):
    # "no change" is 1.0; range [0.1, 1.9] for levels <= 10, floored at 0.1 above that
    return max(0.1, 1.0 + _neg(lvl / _MAX * 0.9))


def color(img, lvl, hp):
    return ImageEnhance.Color(img).enhance(_enh_level(lvl))


def contrast(img, lvl, hp):
    return ImageEnhance.Contrast(img).enhance(_enh_level(lvl))


def brightness(img, lvl, hp):
    return ImageEnhance.Brightness(img).enhance(_enh_level(lvl))


def sharpness(img, lvl, hp):
    return ImageEnhance.Sharpness(img).enhance(_enh_level(lvl))


def color_inc(img, lvl, hp):
    return ImageEnhance.Color(img).enhance(_enh_inc_level(lvl))


def contrast_inc(img, lvl, hp):
    return ImageEnhance.Contrast(img).enhance(_enh_inc_level(lvl))


def brightness_inc(img, lvl, hp):
    return ImageEnhance.Brightness(img).enhance(_enh_inc_level(lvl))


def sharpness_inc(img, lvl, hp):
    return ImageEnhance.Sharpness(img).enhance(_enh_inc_level(lvl))


def shear_x(img, lvl, hp):
    return _affine(img, (1, _neg(lvl / _MAX * 0.3), 0, 0, 1, 0), hp)


def shear_y(img, lvl, hp):
    return _affine(img, (1, 0, 0, _neg(lvl / _MAX * 0.3), 1, 0), hp)


def translate_x_abs(img, lvl, hp):
    return _affine(img, (1, 0, _neg(lvl / _MAX * hp.get("translate_const", 250)), 0, 1, 0), hp)


def translate_y_abs(img, lvl, hp):
    return _affine(img, (1, 0, 0, 0, 1, _neg(lvl / _MAX * hp.get("translate_const", 250))), hp)


def translate_x_rel(img, lvl, hp):
    px = _neg(lvl / _MAX * hp.get("translate_pct", 0.45)) * img.size[0]
    return _affine(img, (1, 0, px, 0, 1, 0), hp)


def translate_y_rel(img, lvl, hp):
    px = _neg(lvl / _MAX * hp.get("translate_pct", 0.45)) * img.size[1]
    return _affine(img, (1, 0, 0, 0, 1, px), hp)


NAME_TO_OP = {
    "AutoContrast": auto_contrast, "Equalize": equalize, "Invert": invert, "Rotate": rotate,
    "Posterize": posterize, "PosterizeIncreasing": posterize_increasing, "PosterizeOriginal": posterize_original,
    "Solarize": solarize, "SolarizeIncreasing": solarize_increasing, "SolarizeAdd": solarize_add,
    "Color": color, "ColorIncreasing": color_inc, "Contrast": contrast, "ContrastIncreasing": contrast_inc,
    "Brightness": brightness, "BrightnessIncreasing": brightness_inc, "Sharpness": sharpness,
    "SharpnessIncreasing": sharpness_inc, "ShearX": shear_x, "ShearY": shear_y, "TranslateX": translate_x_abs,
    "TranslateY": translate_y_abs, "TranslateXRel": translate_x_rel, "TranslateYRel": translate_y_rel,
}

RAND_TRANSFORMS = ["AutoContrast", "Equalize", "Invert", "Rotate", "Posterize", "Solarize", "SolarizeAdd", "Color",
                   "Contrast", "Brightness", "Sharpness", "ShearX", "ShearY", "TranslateXRel", "TranslateYRel"]
RAND_INCREASING_TRANSFORMS = ["AutoContrast", "Equalize", "Invert", "Rotate", "PosterizeIncreasing",
                              "SolarizeIncreasing", "SolarizeAdd", "ColorIncreasing", "ContrastIncreasing",
                              "BrightnessIncreasing", "SharpnessIncreasing", "ShearX", "ShearY", "TranslateXRel",
                              "TranslateYRel"]
AUGMIX_TRANSFORMS = ["AutoContrast", "ColorIncreasing", "ContrastIncreasing", "BrightnessIncreasing",
                     "SharpnessIncreasing", "Equalize", "Rotate", "PosterizeIncreasing", "SolarizeIncreasing",
                     "ShearX", "ShearY", "TranslateXRel", "TranslateYRel"]


class AugmentOp:
    def __init__(self, name, prob=0.5, magnitude=10, hparams=None):
        self.name, self.fn = name, NAME_TO_OP[name]
        self.prob, self.magnitude = prob, magnitude
        self.hp = dict(hparams or {})
        self.mstd = self.hp.get("magnitude_std", 0.0)
        self.mmax = self.hp.get("magnitude_max", _MAX)

    def __call__(self, img):
        if self.prob < 1.0 and random.random() > self.prob:
            return img
        m = self.magnitude
        if self.mstd > 0:
            m = random.uniform(0, m) if self.mstd == float("inf") else random.gauss(m, self.mstd)
        m = max(0.0, min(m, self.mmax))
        return self.fn(img, m, self.hp)


def _parse(spec: str):
    parts = spec.split("-")
    return parts[0], parts[1:]


class RandAugment:
    def __init__(self, ops, num_layers=2):
        self.ops, self.n = ops, num_layers

    def __call__(self, img):
        for op in random.choices(self.ops, k=self.n):
            img = op(img)
        return img


def rand_augment_transform(spec: str, hparams: dict) -> RandAugment:
    name, args = _parse(spec)
    assert name == "rand", spec
    m, n, p, inc = 10.0, 2, 0.5, False
    hp = dict(hparams)
    for a in args:
        if a.startswith("mstd"):
            hp["magnitude_std"] = float(a[4:])
        elif a.startswith("mmax"):
            hp["magnitude_max"] = float(a[4:])
        elif a.startswith("inc"):
            inc = bool(int(a[3:]))
        elif a.startswith("m"):
            m = float(a[1:])
        elif a.startswith("n"):
            n = int(a[1:])
        elif a.startswith("p"):
            p = float(a[1:])
    names = RAND_INCREASING_TRANSFORMS if inc else RAND_TRANSFORMS
    return RandAugment([AugmentOp(x, p, m, hp) for x in names], n)


class AugMix:
    """AugMix (Hendrycks et al. 2020) as timm composes it: ``width`` chains of ``depth`` (or 1-3)
    ops mixed with Dirichlet(alpha) weights, then blended with the original by m ~ Beta(alpha,
    alpha).  ``blended`` mode instead alpha-blends each chain into the running image with weights
    rescaled so the final composite has the same mixing proportions."""

    def __init__(self, ops, alpha=1.0, width=3, depth=-1, blended=False):
        self.ops, self.alpha, self.width, self.depth, self.blended = ops, alpha, width, depth, blended

    def _chain(self, img):
        d = self.depth if self.depth > 0 else random.randint(1, 3)
        for op in random.choices(self.ops, k=d):
            img = op(img)
        return img

    @staticmethod
    def blended_weights(ws, m):
        """Per-step blend alphas a_k (applied last-to-first) such that sequential
        ``img = (1-a_k) img + a_k chain_k`` leaves weight m*w_k on chain k."""
        ws = np.asarray(ws, np.float64) * m
        rest, out = 1.0, []
        for w in ws[::-1]:
            a = w / rest
            rest *= 1.0 - a
            out.append(a)
        return np.asarray(out[::-1], np.float32)

    def __call__(self, img):
        ws = np.random.dirichlet([self.alpha] * self.width).astype(np.float32)
        m = float(np.float32(np.random.beta(self.alpha, self.alpha)))
        if self.blended:
            orig = img
            for a in self.blended_weights(ws, m):
                img = Image.blend(img, self._chain(orig), float(a))
            return img
        mixed = np.zeros(np.asarray(img).shape, dtype=np.float32)
        for w in ws:
            mixed += w * np.asarray(self._chain(img), dtype=np.float32)
        mixed = Image.fromarray(np.clip(mixed, 0, 255).astype(np.uint8))
        return Image.blend(img, mixed, m)


def augmix_transform(spec: str, hparams: dict) -> AugMix:
    name, args = _parse(spec)
    assert name == "augmix", spec
    m, w, d, alpha, blended = 3.0, 3, -1, 1.0, False
    hp = dict(hparams)
    hp.setdefault("magnitude_std", float("inf"))
    i = 0
    while i < len(args):
        a = args[i]
        if a.startswith("mstd"):
            hp["magnitude_std"] = float(a[4:])
        elif a.startswith("m"):
            m = float(a[1:])
        elif a.startswith("w"):
            w = int(a[1:])
        elif a == "d" and i + 1 < len(args):  # "d-1"
            d = -int(args[i + 1])
            i += 1
        elif a.startswith("d"):
            d = int(a[1:])
        elif a.startswith("a"):
            alpha = float(a[1:])
        elif a.startswith("b"):
            blended = bool(int(a[1:]))
        i += 1
    return AugMix([AugmentOp(x, 1.0, m, hp) for x in AUGMIX_TRANSFORMS], alpha, w, d, blended)


# AutoAugment ImageNet policy (Cubuk et al. 2019), (op, prob, magnitude) pairs
POLICY_ORIGINAL = [
    [("PosterizeOriginal", 0.4, 8), ("Rotate", 0.6, 9)], [("Solarize", 0.6, 5), ("AutoContrast", 0.6, 5)],
    [("Equalize", 0.8, 8), ("Equalize", 0.6, 3)], [("PosterizeOriginal", 0.6, 7), ("PosterizeOriginal", 0.6, 6)],
    [("Equalize", 0.4, 7), ("Solarize", 0.2, 4)], [("Equalize", 0.4, 4), ("Rotate", 0.8, 8)],
    [("Solarize", 0.6, 3), ("Equalize", 0.6, 7)], [("PosterizeOriginal", 0.8, 5), ("Equalize", 1.0, 2)],
    [("Rotate", 0.2, 3), ("Solarize", 0.6, 8)], [("Equalize", 0.6, 8), ("PosterizeOriginal", 0.4, 6)],
    [("Rotate", 0.8, 8), ("Color", 0.4, 0)], [("Rotate", 0.4, 9), ("Equalize", 0.6, 2)],
    [("Equalize", 0.0, 7), ("Equalize", 0.8, 8)], [("Invert", 0.6, 4), ("Equalize", 1.0, 8)],
    [("Color", 0.6, 4), ("Contrast", 1.0, 8)], [("Rotate", 0.8, 8), ("Color", 1.0, 2)],
    [("Color", 0.8, 8), ("Solarize", 0.8, 7)], [("Sharpness", 0.4, 7), ("Invert", 0.6, 8)],
    [("ShearX", 0.6, 5), ("Equalize", 1.0, 9)], [("Color", 0.4, 0), ("Equalize", 0.6, 3)],
    [("Equalize", 0.4, 7), ("Solarize", 0.2, 4)], [("Solarize", 0.6, 5), ("AutoContrast", 0.6, 5)],
    [("Invert", 0.6, 4), ("Equalize", 1.0, 8)], [("Color", 0.6, 4), ("Contrast", 1.0, 8)],
    [("Equalize", 0.8, 8), ("Equalize", 0.6, 3)],
]


# ImageNet "v0" policy of the EfficientNet TPU reference implementation (timm ``v0``)
POLICY_V0 = [
    [("Equalize", 0.8, 1), ("ShearY", 0.8, 4)], [("Color", 0.4, 9), ("Equalize", 0.6, 3)],
    [("Color", 0.4, 1), ("Rotate", 0.6, 8)], [("Solarize", 0.8, 3), ("Equalize", 0.4, 7)],
    [("Solarize", 0.4, 2), ("Solarize", 0.6, 2)], [("Color", 0.2, 0), ("Equalize", 0.8, 8)],
    [("Equalize", 0.4, 8), ("SolarizeAdd", 0.8, 3)], [("ShearX", 0.2, 9), ("Rotate", 0.6, 8)],
    [("Color", 0.6, 1), ("Equalize", 1.0, 2)], [("Invert", 0.4, 9), ("Rotate", 0.6, 0)],
    [("Equalize", 1.0, 9), ("ShearY", 0.6, 3)], [("Color", 0.4, 7), ("Equalize", 0.6, 0)],
    [("Posterize", 0.4, 6), ("AutoContrast", 0.4, 7)], [("Solarize", 0.6, 8), ("Color", 0.6, 9)],
    [("Solarize", 0.2, 4), ("Rotate", 0.8, 9)], [("Rotate", 1.0, 7), ("TranslateYRel", 0.8, 9)],
    [("ShearX", 0.0, 0), ("Solarize", 0.8, 4)], [("ShearY", 0.8, 0), ("Color", 0.6, 4)],
    [("Color", 1.0, 0), ("Rotate", 0.6, 2)], [("Equalize", 0.8, 4), ("Equalize", 0.0, 8)],
    [("Equalize", 1.0, 4), ("AutoContrast", 0.6, 2)], [("ShearY", 0.4, 7), ("SolarizeAdd", 0.6, 7)],
    [("Posterize", 0.8, 2), ("Solarize", 0.6, 10)], [("Solarize", 0.6, 8), ("Equalize", 0.6, 1)],
    [("Color", 0.8, 6), ("Rotate", 0.4, 5)],
]


def _r_variant(policy):
    """The ``...r`` policies: Posterize replaced by the increasing-severity PosterizeIncreasing."""
    sub = {"Posterize": "PosterizeIncreasing", "PosterizeOriginal": "PosterizeIncreasing"}
    return [[(sub.get(n, n), p, m) for n, p, m in sp] for sp in policy]


POLICIES = {"original": POLICY_ORIGINAL, "originalr": _r_variant(POLICY_ORIGINAL),
            "v0": POLICY_V0, "v0r": _r_variant(POLICY_V0)}


class AutoAugment:
    def __init__(self, policy):
        self.policy = policy

    def __call__(self, img):
        for op in random.choice(self.policy):
            img = op(img)
        return img


def auto_augment_transform(spec: str, hparams: dict) -> AutoAugment:
    name, args = _parse(spec)
    hp = dict(hparams)
    for a in args:
        if a.startswith("mstd"):
            hp["magnitude_std"] = float(a[4:])
    if name not in POLICIES:
        raise ValueError(f"unknown AutoAugment policy {spec}")
    return AutoAugment([[AugmentOp(n, p, m, hp) for n, p, m in sp] for sp in POLICIES[name]])
