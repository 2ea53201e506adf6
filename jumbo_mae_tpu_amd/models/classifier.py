"""Finetune / linear-probe task module.

Parity: ``FinetuneModule`` (/root/reference/src/finetuning.py:78-106), ``CRITERION_COLLECTION``
(:39-42), the classifier branch of ``ViT.__call__`` (modeling.py:268-274) and ``validation_step``
(finetuning.py:157-165).

* labels: int -> one-hot; training applies label smoothing then Mixup/CutMix;
* logits = head(LN(x)[:, :3].reshape(B, 3D)) -- only the 3 CLS rows go through the final LN
  (per-row op, identical result);
* linear probing: the encoder runs without autograd (== ``stop_gradient``) and the head is
  SyncBatchNorm + Dense;
* accuracy = membership of the top-1 / top-5 predictions in the arg-max label set.
Fixes: RNG streams advance every step (quirk Q4); validation loss is the true per-sample masked
mean (the reference multiplies the batch-mean loss, padded samples included, by the valid count).
"""

from __future__ import annotations

import torch
import torch.nn.functional as F

from ..config import ViTConfig
from ..ops import functional as Fn
from ..ops import mae as mae_ops
from ..utils.mixup import Mixup, smooth_labels
from .params import ParamStore
from .vit import JumboViT, LinearCLS


def softmax_cross_entropy(logits, labels):
    return -(labels * F.log_softmax(logits, -1)).sum(-1)


def sigmoid_bce(logits, labels):
    t = (labels > 0).to(logits.dtype)
    return F.binary_cross_entropy_with_logits(logits, t, reduction="none").mean(-1)


CRITERION_COLLECTION = {"ce": softmax_cross_entropy, "bce": sigmoid_bce}


def _capturing() -> bool:
    return torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()


class FinetuneModel:
    def __init__(self, cfg: ViTConfig, mixup: Mixup | None = None, label_smoothing: float = 0.0,
                 criterion: str = "ce", group=None):
        assert cfg.labels > 0
        self.cfg = cfg
        self.store = ParamStore()
        s = self.store
        trainable_encoder = not cfg.linear_probing
        self.encoder = JumboViT(s, cfg, ("model",), trainable=trainable_encoder)
        self.head = LinearCLS(s, ("model", "head"), cfg.jumbo_dim, cfg.labels, cfg.batch_norm)
        self.mixup = mixup or Mixup(0.0, 0.0)
        self.label_smoothing = label_smoothing if criterion == "ce" else 0.0
        self.criterion = CRITERION_COLLECTION[criterion]
        self.group = group

    def to(self, device, compute_dtype=torch.float32, seed: int = 0):
        g = torch.Generator(device=device).manual_seed(seed)
        self.store.finalize(device, compute_dtype, g)
        self.head.init_stats(device)
        return self

    @property
    def device(self):
        return self.store.master.device

    # ---------------------------------------------------------------- pieces
    micro_index = 0

    def prepare_step(self, i: int, images_u8, labels=None) -> None:
        """Host part of a train step (engine.Trainer.host_prepare): draw micro-batch ``i``'s Mixup /
        CutMix decision; its device buffers are what the (possibly graph-replayed) forward reads."""
        if not self.mixup.active:
            return
        if not hasattr(self, "_plans"):
            self._plans = {}
        B, _, H, W = images_u8.shape
        self._plans[i] = self.mixup.plan(B, H, W, images_u8.device, tag=str(i))

    def patches(self, images_u8, labels, rngs, det):
        """(patch rows [B*N, p*p*3] in the compute dtype, labels) -- Mixup / CutMix applied when
        training (one plan per batch; the blend is fused into the patch gather on the GPU)."""
        B, _, H, W = images_u8.shape
        plan = None
        if not det and self.mixup.active:
            plans = getattr(self, "_plans", {})
            plan = plans.pop(self.micro_index, None) if not _capturing() else plans.get(self.micro_index)
            if plan is None:  # direct forward call without a prepared step: draw here
                plan = self.mixup.plan(B, H, W, images_u8.device, rngs.get("mixup") if rngs else None)
        if labels is not None:
            labels = Mixup.mix_labels(labels, plan)
        rows = mae_ops.mixed_patches(images_u8, plan, self.cfg.patch_size, self.store.compute_dtype)
        return rows, labels

    def features(self, rows, B, rngs=None, det=True):
        cfg = self.cfg
        drop = rngs.get("dropout") if rngs else None
        x = self.encoder.embed_rows(rows, None, B)
        x = self.encoder.blocks(x, drop, det)
        C = cfg.num_cls_tokens
        h = Fn.layer_norm(x[:, :C], self.encoder.norm.g, self.encoder.norm.b, torch.float32)
        return h.reshape(B, C * cfg.dim)

    def logits(self, images_u8, labels=None, rngs=None, det=True):
        B = images_u8.shape[0]
        rows, labels = self.patches(images_u8, labels, rngs, det)
        if self.cfg.linear_probing:
            with torch.no_grad():
                feats = self.features(rows, B, rngs, det)
        else:
            feats = self.features(rows, B, rngs, det)
        return self.head(feats, det, self.group), labels

    # ---------------------------------------------------------------- train / eval
    def forward(self, images_u8, labels, rngs=None, det=False):
        labels = self._prep_labels(labels)
        if not det:
            labels = smooth_labels(labels, self.label_smoothing)
        logits, labels = self.logits(images_u8, labels, rngs, det)
        loss = self.criterion(logits, labels).mean()
        acc1, acc5 = self.accuracy(logits, labels)
        return {"loss": loss, "acc1": acc1.float().mean(), "acc5": acc5.float().mean()}

    __call__ = forward

    def _prep_labels(self, labels):
        if labels.dim() == 1:  # one-hot by scatter: F.one_hot validates the range with a host sync
            idx = labels.long().clamp(0, self.cfg.labels - 1).view(-1, 1)
            return torch.zeros(labels.shape[0], self.cfg.labels, device=labels.device).scatter_(1, idx, 1.0)
        return labels.float()

    @staticmethod
    def accuracy(logits, labels):
        lab = labels == labels.max(-1, keepdim=True).values
        k = min(5, logits.shape[-1])
        top = logits.topk(k, -1).indices
        accs = torch.gather(lab, 1, top)
        return accs[:, 0], accs.any(-1)

    @torch.no_grad()
    def evaluate(self, images_u8, labels, rngs=None) -> dict:
        """Sums over valid (label != -1) samples, like validation_step (finetuning.py:157-165)."""
        valid = (labels != -1)
        lab = self._prep_labels(torch.where(valid, labels, torch.zeros_like(labels)))
        logits, _ = self.logits(images_u8, lab, rngs, det=True)
        loss = self.criterion(logits, lab)
        acc1, acc5 = self.accuracy(logits, lab)
        v = valid.float()
        return {"loss": (loss * v).sum(), "acc1": (acc1.float() * v).sum(), "acc5": (acc5.float() * v).sum(),
                "num_samples": v.sum()}

    # ---------------------------------------------------------------- params
    def flax_params(self) -> dict:
        return self.store.to_flax_tree()

    def batch_stats(self) -> dict | None:
        if not self.cfg.batch_norm:
            return None
        return {"model": {"head": {"BatchNorm_0": {"mean": self.head.running_mean.cpu().numpy(),
                                                   "var": self.head.running_var.cpu().numpy()}}}}
