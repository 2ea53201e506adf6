"""Flax tree <-> PyTorch (timm-style) state dict conversion, Jumbo-aware.

Reference: scripts/convert_flax_to_pytorch.py:25-91 and scripts/convert_pytorch_to_flax.py:24-100.
Those scripts target the upstream single-CLS layout and ignore the Jumbo leaves (quirk Q9).
Here the standard ViT parts keep timm names (``patch_embed.proj``, ``blocks.i.attn.qkv``,
``blocks.i.mlp.fc1`` ...) and the Jumbo parts get explicit names:

  model/cls_tokens (1,3,D)            -> cls_tokens        (and cls_token = cls_tokens[:, :1])
  model/embed/wpe (g,g,D) | sincos    -> pos_embed (1, 3 + g*g, D) (zero CLS slots, like the
                                         reference converter's single padded slot)
  model/jumbo_mlp/w{1,2}              -> jumbo_mlp.fc{1,2}.{weight,bias}
  model/layer_i/norm3                 -> blocks.i.norm3.{weight,bias}
  model/layer_i/scale{1,2,3}          -> blocks.i.ls{1,2,3}.gamma
  model/head/Dense_0                  -> head.{weight,bias}
  model/head/BatchNorm_0              -> head_bn.{weight,bias}
"""

from __future__ import annotations

import re

import numpy as np

from ..utils.posemb import _sincos2d_np


def _t(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.float32))


def flax_to_torch(params: dict, exclude_heads: bool = False, num_cls: int = 3, image_size: int = 224) -> dict:
    """``image_size`` sets the patch grid of a sincos model (no learnable table in the tree): the
    exported ``pos_embed`` is the fixed table of an ``image_size`` input."""
    m = params["model"] if "model" in params else params
    emb = m["embed"]
    D = emb["wte"]["bias"].shape[0]
    sd = {}
    cls = _t(m["cls_tokens"]) if "cls_tokens" in m else _t(m.get("embed", {}).get("cls_token", np.zeros((1, 1, D))))
    sd["cls_tokens"] = cls
    sd["cls_token"] = cls[:, :1]
    if "wpe" in emb:
        pos = _t(emb["wpe"])
        g = pos.shape[0]
    else:
        k = emb["wte"]["kernel"]
        g = image_size // k.shape[0]  # HWIO kernel: k.shape[0] is the patch size
        pos = _sincos2d_np(g, g, D)
    pos = pos.reshape(1, -1, D)
    sd["pos_embed"] = np.concatenate([np.zeros((1, cls.shape[1], D), np.float32), pos], 1)
    sd["patch_embed.proj.weight"] = _t(emb["wte"]["kernel"]).transpose(3, 2, 0, 1).copy()
    sd["patch_embed.proj.bias"] = _t(emb["wte"]["bias"])
    if "norm" in m:
        sd["norm.weight"] = _t(m["norm"]["scale"])
        sd["norm.bias"] = _t(m["norm"]["bias"])
    if "jumbo_mlp" in m:
        for i, n in ((1, "w1"), (2, "w2")):
            sd[f"jumbo_mlp.fc{i}.weight"] = _t(m["jumbo_mlp"][n]["kernel"]).T.copy()
            sd[f"jumbo_mlp.fc{i}.bias"] = _t(m["jumbo_mlp"][n]["bias"])
    if "head" in m and not exclude_heads:
        h = m["head"]
        dense = h["Dense_0"] if "Dense_0" in h else h
        sd["head.weight"] = _t(dense["kernel"]).T.copy()
        sd["head.bias"] = _t(dense["bias"])
        if "BatchNorm_0" in h:
            sd["head_bn.weight"] = _t(h["BatchNorm_0"]["scale"])
            sd["head_bn.bias"] = _t(h["BatchNorm_0"]["bias"])
    for name, layer in m.items():
        mm = re.fullmatch(r"layer_(\d+)", name)
        if not mm:
            continue
        i = int(mm.group(1))
        a = layer["attn"]
        wq, wk, wv = (_t(a[n]["kernel"]).reshape(D, -1) for n in ("wq", "wk", "wv"))
        sd[f"blocks.{i}.attn.qkv.weight"] = np.concatenate([wq, wk, wv], 1).T.copy()
        sd[f"blocks.{i}.attn.qkv.bias"] = np.concatenate([_t(a[n]["bias"]).reshape(-1) for n in ("wq", "wk", "wv")])
        sd[f"blocks.{i}.attn.proj.weight"] = _t(a["wo"]["kernel"]).reshape(-1, D).T.copy()
        sd[f"blocks.{i}.attn.proj.bias"] = _t(a["wo"]["bias"])
        for j, n in ((1, "w1"), (2, "w2")):
            sd[f"blocks.{i}.mlp.fc{j}.weight"] = _t(layer["ff"][n]["kernel"]).T.copy()
            sd[f"blocks.{i}.mlp.fc{j}.bias"] = _t(layer["ff"][n]["bias"])
        for nn_ in ("norm1", "norm2", "norm3"):
            if nn_ in layer:
                sd[f"blocks.{i}.{nn_}.weight"] = _t(layer[nn_]["scale"])
                sd[f"blocks.{i}.{nn_}.bias"] = _t(layer[nn_]["bias"])
        for j in (1, 2, 3):
            if f"scale{j}" in layer:
                sd[f"blocks.{i}.ls{j}.gamma"] = _t(layer[f"scale{j}"])
    return sd


def torch_to_flax(sd: dict, num_heads: int, exclude_heads: bool = False, learnable_posemb: bool = True) -> dict:
    """Inverse of ``flax_to_torch`` (``convert_pytorch_to_flax.py`` behaviour, Jumbo-aware).

    Single-CLS timm checkpoints are accepted: ``cls_token`` is tiled to three CLS tokens and the
    CLS slot of ``pos_embed`` is folded in (reference ``:35``); missing Jumbo leaves are skipped
    (the caller keeps their fresh initialisation).
    """
    sd = {k: np.asarray(v, dtype=np.float32) for k, v in sd.items()}
    w = sd["patch_embed.proj.weight"]
    D = w.shape[0]
    hd = D // num_heads
    m: dict = {"embed": {"wte": {"kernel": w.transpose(2, 3, 1, 0).copy(), "bias": sd["patch_embed.proj.bias"]}}}
    if "cls_tokens" in sd:
        cls = sd["cls_tokens"]
    else:
        cls = np.repeat(sd["cls_token"], 3, axis=1)
    ncls = cls.shape[1]
    if "pos_embed" in sd:
        pos = sd["pos_embed"]
        n = pos.shape[1]
        g = int(round((n - ncls) ** 0.5))
        if g * g == n - ncls:
            cls = cls + pos[:, :ncls]
            pos = pos[:, ncls:]
        else:  # single-slot timm layout
            g = int(round((n - 1) ** 0.5))
            cls = cls + pos[:, :1]
            pos = pos[:, 1:]
        if learnable_posemb:
            m["embed"]["wpe"] = pos.reshape(g, g, D)
    m["cls_tokens"] = cls
    if "norm.weight" in sd:
        m["norm"] = {"scale": sd["norm.weight"], "bias": sd["norm.bias"]}
    if "jumbo_mlp.fc1.weight" in sd:
        m["jumbo_mlp"] = {f"w{j}": {"kernel": sd[f"jumbo_mlp.fc{j}.weight"].T.copy(),
                                    "bias": sd[f"jumbo_mlp.fc{j}.bias"]} for j in (1, 2)}
    if "head.weight" in sd and not exclude_heads:
        head = {"Dense_0": {"kernel": sd["head.weight"].T.copy(), "bias": sd["head.bias"]}}
        if "head_bn.weight" in sd:
            head["BatchNorm_0"] = {"scale": sd["head_bn.weight"], "bias": sd["head_bn.bias"]}
        m["head"] = head
    idx = sorted({int(k.split(".")[1]) for k in sd if k.startswith("blocks.")})
    for i in idx:
        p = f"blocks.{i}."
        qkv = sd[p + "attn.qkv.weight"].T  # (D, 3D)
        qkvb = sd[p + "attn.qkv.bias"]
        attn = {}
        for j, n in enumerate(("wq", "wk", "wv")):
            attn[n] = {"kernel": qkv[:, j * D:(j + 1) * D].reshape(D, num_heads, hd).copy(),
                       "bias": qkvb[j * D:(j + 1) * D].reshape(num_heads, hd).copy()}
        attn["wo"] = {"kernel": sd[p + "attn.proj.weight"].T.reshape(num_heads, hd, D).copy(),
                      "bias": sd[p + "attn.proj.bias"]}
        layer = {"attn": attn,
                 "ff": {f"w{j}": {"kernel": sd[p + f"mlp.fc{j}.weight"].T.copy(), "bias": sd[p + f"mlp.fc{j}.bias"]}
                        for j in (1, 2)}}
        for nn_ in ("norm1", "norm2", "norm3"):
            if p + nn_ + ".weight" in sd:
                layer[nn_] = {"scale": sd[p + nn_ + ".weight"], "bias": sd[p + nn_ + ".bias"]}
        for j in (1, 2, 3):
            for key in (p + f"ls{j}.gamma", p + f"ls{j}.weight"):
                if key in sd:
                    layer[f"scale{j}"] = sd[key]
        m[f"layer_{i}"] = layer
    return {"model": m}
