"""Model hyper-parameter records.

Parity: ``ViTBase`` / ``MAEDecoderBase`` of the reference
(/root/reference/src/modeling.py:35-104).  Derived quantities (``head_dim``,
``hidden_dim = 4*dim``, ``num_patches``) follow the reference exactly; the
decoder record exposes the same fields with the ``dec_`` prefix.
"""

from __future__ import annotations

from dataclasses import asdict, dataclass, field
from typing import Literal

NUM_CLS_TOKENS = 3  # jumbo: three CLS tokens concatenated into one 3*dim token (modeling.py:170,222)


@dataclass
class ViTConfig:
    layers: int = 12
    dim: int = 768
    heads: int = 12
    labels: int = 1000  # <=0 -> MAE mode (no head), modeling.py:239-241
    layerscale: bool = False

    patch_size: int = 16
    image_size: int = 224
    posemb: Literal["learnable", "sincos2d"] = "learnable"
    pooling: Literal["cls", "gap"] = "cls"  # accepted for CLI parity, unused (modeling.py:272)

    dropout: float = 0.0
    droppath: float = 0.0
    grad_ckpt: bool = False

    image_mask_ratio: float | None = 0.75
    linear_probing: bool = False
    batch_norm: bool = False
    num_cls_tokens: int = NUM_CLS_TOKENS

    @property
    def head_dim(self) -> int:
        return self.dim // self.heads

    @property
    def hidden_dim(self) -> int:
        return 4 * self.dim

    @property
    def jumbo_dim(self) -> int:
        return self.dim * self.num_cls_tokens

    @property
    def grid(self) -> int:
        return self.image_size // self.patch_size

    @property
    def num_patches(self) -> tuple[int, int]:
        return (self.grid, self.grid)

    @property
    def seq_patches(self) -> int:
        return self.grid * self.grid

    @property
    def keep_len(self) -> int:
        """Patch tokens kept by random masking: int(N*(1-ratio)) (modeling.py:255)."""
        if self.image_mask_ratio is None:
            return self.seq_patches
        return int(self.seq_patches * (1.0 - self.image_mask_ratio))

    def as_dict(self) -> dict:
        return asdict(self)


@dataclass
class DecoderConfig:
    dec_layers: int = 6
    dec_dim: int = 512
    dec_heads: int = 8
    dec_layerscale: bool = False
    dec_posemb: Literal["learnable", "sincos2d"] = "learnable"  # ignored by the reference (Q10)
    dec_dropout: float = 0.0
    dec_droppath: float = 0.0
    grad_ckpt: bool = False
    patch_size: int = 16
    image_size: int = 224

    @property
    def head_dim(self) -> int:
        return self.dec_dim // self.dec_heads

    @property
    def hidden_dim(self) -> int:
        return 4 * self.dec_dim

    @property
    def grid(self) -> int:
        return self.image_size // self.patch_size

    @property
    def num_patches(self) -> tuple[int, int]:
        return (self.grid, self.grid)


# Named presets (the reference selects sizes through CLI flags; these are conveniences).
PRESETS: dict[str, dict] = {
    "vit_tiny_patch16": dict(layers=12, dim=192, heads=3),
    "vit_small_patch16": dict(layers=12, dim=384, heads=6),
    "vit_base_patch16": dict(layers=12, dim=768, heads=12),
    "vit_large_patch16": dict(layers=24, dim=1024, heads=16),
    "vit_huge_patch14": dict(layers=32, dim=1280, heads=16, patch_size=14),
}

MAE_DECODER_DEFAULT = dict(dec_layers=8, dec_dim=512, dec_heads=16)


def vit_config(name: str, **overrides) -> ViTConfig:
    kw = dict(PRESETS[name])
    kw.update(overrides)
    return ViTConfig(**kw)


def decoder_config(**overrides) -> DecoderConfig:
    kw = dict(MAE_DECODER_DEFAULT)
    kw.update(overrides)
    return DecoderConfig(**kw)


@dataclass
class RunShape:
    """Static per-rank shapes of a pretrain step (used by bench and HIP-graph capture)."""

    batch: int
    image_size: int = 224
    extra: dict = field(default_factory=dict)
