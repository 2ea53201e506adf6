"""Batch-level Mixup / CutMix and label smoothing.

Reference: ``Mixup`` (/root/reference/src/utils.py:66-111) and ``optax.smooth_labels``
(finetuning.py:94).  Semantics kept: one ``lambda ~ Beta(a, a)`` and one permutation per batch
(per rank); CutMix box side ``sqrt(1 - lambda)`` centred at a uniform point, evaluated on a
``linspace(0, 1, W|H)`` grid (so the kept area, not lambda, weights the labels); when both are
enabled each batch picks one of the two with probability 1/2.  The permutation / blend run on
the device; the handful of batch-level scalars are drawn from a per-rank host generator.
Images are NCHW here (the reference is NHWC; the box mask is transposed accordingly).
"""

from __future__ import annotations

import numpy as np
import torch


def smooth_labels(labels: torch.Tensor, alpha: float) -> torch.Tensor:
    """optax.smooth_labels: (1 - alpha) * labels + alpha / num_classes."""
    if alpha == 0:
        return labels
    return (1.0 - alpha) * labels + alpha / labels.shape[-1]


class Mixup:
    def __init__(self, mixup_alpha: float = 0.8, cutmix_alpha: float = 1.0, seed: int = 0):
        self.mixup_alpha = mixup_alpha
        self.cutmix_alpha = cutmix_alpha
        self.rs = np.random.default_rng(seed)

    @property
    def active(self) -> bool:
        return self.mixup_alpha > 0 or self.cutmix_alpha > 0

    def _perm(self, n, device, gen):
        return torch.randperm(n, device=device, generator=gen)

    def apply_mixup(self, images, labels, gen=None):
        ratio = float(self.rs.beta(self.mixup_alpha, self.mixup_alpha))
        perm = self._perm(images.shape[0], images.device, gen)
        images = ratio * images + (1 - ratio) * images[perm]
        labels = ratio * labels + (1 - ratio) * labels[perm]
        return images, labels

    def random_bounding_box(self, ratio: float, width: int, height: int, device) -> torch.Tensor:
        size = (1 - ratio) ** 0.5
        xstart, ystart = self.rs.uniform(size=2)
        xr = torch.linspace(0, 1, width, device=device)
        yr = torch.linspace(0, 1, height, device=device)
        xm = (xstart - 0.5 * size <= xr) & (xr < xstart + 0.5 * size)
        ym = (ystart - 0.5 * size <= yr) & (yr < ystart + 0.5 * size)
        return ~(ym[:, None] & xm[None, :])  # [H, W], True = keep own image

    def apply_cutmix(self, images, labels, gen=None):
        ratio = float(self.rs.beta(self.cutmix_alpha, self.cutmix_alpha))
        H, W = images.shape[-2:]
        m = self.random_bounding_box(ratio, W, H, images.device).to(images.dtype)
        label_w = m.mean()
        perm = self._perm(images.shape[0], images.device, gen)
        images = m * images + (1 - m) * images[perm]
        labels = label_w * labels + (1 - label_w) * labels[perm]
        return images, labels

    def __call__(self, images, labels, gen=None):
        if self.mixup_alpha == 0 and self.cutmix_alpha == 0:
            return images, labels
        if self.mixup_alpha > 0 and self.cutmix_alpha == 0:
            return self.apply_mixup(images, labels, gen)
        if self.mixup_alpha == 0 and self.cutmix_alpha > 0:
            return self.apply_cutmix(images, labels, gen)
        if self.rs.uniform() > 0.5:
            return self.apply_mixup(images, labels, gen)
        return self.apply_cutmix(images, labels, gen)
