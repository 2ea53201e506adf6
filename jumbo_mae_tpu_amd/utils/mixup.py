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

    def _perm(self, n, device=None, gen=None):
        """One permutation of the batch per mixed batch, drawn from the host generator (a step's
        host draws all go through the step feeder, so the device work can replay from a graph)."""
        return self.rs.permutation(n)

    # ---------------------------------------------------------------- batch plan
    def plan(self, batch: int, height: int, width: int, device, gen=None, tag: str = "") -> dict | None:
        """Draw this batch's mixing decision (same RNG consumption order as the reference's
        Mixup.__call__): ``{"mode": "mixup"|"cutmix", "ratio", "perm", "box", "label_w"}`` where
        ``box`` = (y0, y1, x0, x1) is the half-open pixel range taken from the permuted image and
        ``label_w`` the weight of the own label.  On a GPU the decision is also delivered to static
        device buffers (``dev``: params [mode, ratio, label_w], box, perm) through the step
        feeder.  None when mixing is off."""
        if self.mixup_alpha == 0 and self.cutmix_alpha == 0:
            return None
        if self.mixup_alpha > 0 and self.cutmix_alpha > 0:
            mode = "mixup" if self.rs.uniform() > 0.5 else "cutmix"
        else:
            mode = "mixup" if self.mixup_alpha > 0 else "cutmix"
        if mode == "mixup":
            ratio = float(self.rs.beta(self.mixup_alpha, self.mixup_alpha))
            box, label_w = None, ratio
        else:
            ratio = float(self.rs.beta(self.cutmix_alpha, self.cutmix_alpha))
            box = self._box(ratio, width, height)
            y0, y1, x0, x1 = box
            label_w = 1.0 - float((y1 - y0) * (x1 - x0)) / float(height * width)
        perm_np = self._perm(batch)
        plan = {"mode": mode, "ratio": ratio, "box": box, "label_w": label_w}
        device = torch.device(device)
        if device.type == "cuda":
            from ..runtime.feeder import feeder
            f = feeder(device)
            plan["dev"] = {
                "params": f.put("mixup_params" + tag, [1.0 if mode == "mixup" else 2.0, ratio, label_w]),
                "box": f.put("mixup_box" + tag, list(box) if box else [0, 0, 0, 0], dtype=torch.int32),
                "perm": f.put("mixup_perm" + tag, perm_np, dtype=torch.int32),
            }
            plan["perm"] = plan["dev"]["perm"]  # int32, static (indexing casts inside the step)
            plan["label_w_t"] = plan["dev"]["params"][2]
        else:
            plan["perm"] = torch.as_tensor(perm_np, dtype=torch.long)
            plan["label_w_t"] = label_w
        return plan

    def _box(self, ratio: float, width: int, height: int):
        """Pixel ranges of the CutMix box on the reference's linspace(0, 1, W|H) grid
        (evaluated with torch's fp32 linspace so the edges match the mask formulation)."""
        size = (1 - ratio) ** 0.5
        xstart, ystart = self.rs.uniform(size=2)

        def rng(start, n):
            r = torch.linspace(0, 1, n)
            inside = ((start - 0.5 * size <= r) & (r < start + 0.5 * size)).nonzero().flatten()
            if inside.numel() == 0:
                return 0, 0
            return int(inside[0]), int(inside[-1]) + 1

        x0, x1 = rng(xstart, width)
        y0, y1 = rng(ystart, height)
        if x0 == x1 or y0 == y1:
            return 0, 0, 0, 0
        return y0, y1, x0, x1

    @staticmethod
    def mix_labels(labels, plan):
        if plan is None:
            return labels
        w = plan["label_w_t"]  # device scalar on a GPU (no host value enters the step)
        return w * labels + (1 - w) * labels[plan["perm"].long()]

    @staticmethod
    def mix_images(images, plan):
        """NCHW float images mixed per ``plan`` (torch composition; the HIP path fuses this into
        the patch gather, ops/mae.py mixed_patches)."""
        if plan is None:
            return images
        other = images[plan["perm"].long().to(images.device)]
        if plan["mode"] == "mixup":
            r = plan["ratio"]
            return r * images + (1 - r) * other
        y0, y1, x0, x1 = plan["box"]
        H, W = images.shape[-2:]
        keep = torch.ones((H, W), dtype=images.dtype, device=images.device)
        keep[y0:y1, x0:x1] = 0
        return keep * images + (1 - keep) * other

    def __call__(self, images, labels, gen=None):
        plan = self.plan(images.shape[0], images.shape[-2], images.shape[-1], images.device, gen)
        return self.mix_images(images, plan), self.mix_labels(labels, plan)
