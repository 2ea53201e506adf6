"""Jumbo ViT encoder, MAE decoder and classification head on the flat ParamStore.

Parity map (reference /root/reference/src/modeling.py):
  PatchEmbed ............ :106-124  (16x16/16 conv == GEMM over (ph,pw,c)-ordered patches)
  Attention ............. :127-138  (wq|wk|wv fused into one GEMM over adjacent segments)
  FeedForward ........... :141-148
  ViTLayer .............. :150-167  (decoder block)
  JumboLayer ............ :169-206  (encoder block: CLS tokens -> shared jumbo MLP)
  LinearCLS ............. :209-219  (SyncBatchNorm + Dense)
  ViT ................... :221-274  (shared jumbo_mlp built once, passed to every layer)
  MAEDecoder ............ :276-298

Parameter names/shapes are those of the Flax tree so that checkpoints are
interchangeable.  MAE mode is *mask-first*: the random permutation is drawn before the patch
embedding and only the kept patches are embedded (bit-for-bit the same math as embedding all
196 patches and gathering afterwards, 4x fewer patch-embed FLOPs).
"""

from __future__ import annotations

import math
import os

import numpy as np
import torch

from ..config import DecoderConfig, ViTConfig
from ..ops import blocks
from ..ops import dropout as Dr
from ..ops import functional as Fn
from ..ops import mae as mae_ops
from ..utils.posemb import fixed_sincos2d_embeddings
from .params import ParamStore, const_, ones_, trunc_normal_, trunc_normal_t, zeros_


def use_fused_blocks() -> bool:
    """One autograd node per transformer block (ops/blocks.py); JMAE_PER_OP=1 selects the per-op
    autograd graph instead (same kernels, used by tests to cross-check the hand-written backward)."""
    return os.environ.get("JMAE_PER_OP", "0") != "1"


# ------------------------------------------------------------------------- layout helpers
def _dense_kernel(store: ParamStore, path, in_shape, out_shape, trainable=True):
    """Dense/DenseGeneral kernel stored out x in; Flax layout in_shape + out_shape."""
    fin, fout = int(np.prod(in_shape)), int(np.prod(out_shape))
    flax_shape = tuple(in_shape) + tuple(out_shape)
    return store.add(
        path, (fout, fin), trunc_normal_t(0.02), flax_shape=flax_shape,
        to_flax=lambda a, fs=flax_shape: a.T.reshape(fs),
        from_flax=lambda a, fi=fin, fo=fout: a.reshape(fi, fo).T,
        trainable=trainable,
    )


def _bias(store: ParamStore, path, out_shape, trainable=True):
    n = int(np.prod(out_shape))
    return store.add(path, (n,), zeros_, flax_shape=tuple(out_shape),
                     to_flax=lambda a, s=tuple(out_shape): a.reshape(s),
                     from_flax=lambda a, n=n: a.reshape(n), trainable=trainable)


class Dense:
    def __init__(self, store, path, in_dim, out_dim, trainable=True):
        self.k = store.handle(_dense_kernel(store, path + ("kernel",), (in_dim,), (out_dim,), trainable))
        self.b = store.handle(_bias(store, path + ("bias",), (out_dim,), trainable))

    def __call__(self, x, gelu=False):
        return Fn.linear(x, self.k, self.b, gelu=gelu)


class LayerNorm:
    def __init__(self, store, path, dim, trainable=True):
        self.g = store.handle(store.add(path + ("scale",), (dim,), ones_, trainable=trainable))
        self.b = store.handle(store.add(path + ("bias",), (dim,), zeros_, trainable=trainable))

    def __call__(self, x, out_dtype=None, row0: int = 0):
        return Fn.layer_norm(x, self.g, self.b, out_dtype, row0)


class FeedForward:
    """Dense(4*dim) -> gelu(tanh) -> dropout -> Dense(dim) -> dropout (modeling.py:141-148)."""

    def __init__(self, store, path, dim, hidden, dropout=0.0, trainable=True):
        self.w1 = Dense(store, path + ("w1",), dim, hidden, trainable)
        self.w2 = Dense(store, path + ("w2",), hidden, dim, trainable)
        self.dropout = dropout

    def __call__(self, x, rng=None, det=True, seeds=None):
        h = self.w1(x, gelu=True)
        h = _dropout(h, self.dropout, rng, det, seeds and seeds[0])
        y = self.w2(h)
        return _dropout(y, self.dropout, rng, det, seeds and seeds[1])


class Attention:
    """Multi-head self-attention; wq|wk|wv are adjacent segments read as one [3D, D] GEMM."""

    def __init__(self, store, path, dim, heads, dropout=0.0, trainable=True):
        hd = dim // heads
        self.dim, self.heads, self.dropout = dim, heads, dropout
        ks = [_dense_kernel(store, path + (n, "kernel"), (dim,), (heads, hd), trainable) for n in ("wq", "wk", "wv")]
        bs = [_bias(store, path + (n, "bias"), (heads, hd), trainable) for n in ("wq", "wk", "wv")]
        self.qkv_k = store.handle(ks, (3 * dim, dim))
        self.qkv_b = store.handle(bs, (3 * dim,))
        self.wo_k = store.handle(_dense_kernel(store, path + ("wo", "kernel"), (heads, hd), (dim,), trainable))
        self.wo_b = store.handle(_bias(store, path + ("wo", "bias"), (dim,), trainable))

    def __call__(self, x2d, B, S, rng=None, det=True, seeds=None):
        qkv = Fn.linear(x2d, self.qkv_k, self.qkv_b).view(B, S, 3 * self.dim)
        if self.dropout > 0 and not det:
            o = _attention_with_dropout(qkv, self.heads, self.dropout, rng, seeds and seeds[0])
        else:
            o = Fn.attention(qkv, self.heads)
        y = Fn.linear(o.view(B * S, self.dim), self.wo_k, self.wo_b)
        return _dropout(y, self.dropout, rng, det, seeds and seeds[1])


def _dropout(x, rate, rng, det, seed=None):
    """Flax nn.Dropout (train mode): hash-mask HIP kernel, mask regenerated in backward (ops/dropout.py)."""
    if rate <= 0.0 or det:
        return x
    return Dr.dropout(x, rate, rng, seed)


def _layer_seeds(rate, rng, device, det, n):
    """The dropout seeds of one layer from one draw (both paths use the same order: attention
    probabilities, attention output, [jumbo MLP hidden, output,] FF hidden, FF output), or None."""
    if rate <= 0.0 or det or rate >= 1.0:
        return None
    return Dr.draw_seeds(rng, device, n)


def _drops(seeds, rate, jumbo):
    if seeds is None:
        return None
    if jumbo:
        return blocks.Drops(rate, seeds[0], seeds[1], seeds[4], seeds[5], seeds[2], seeds[3])
    return blocks.Drops(rate, *seeds)


def _attention_with_dropout(qkv, heads, rate, rng, seed=None):
    """Attention with dropout on the probabilities (all presets use dropout 0): the two batched
    products on the BLAS library in fp32, softmax + dropout (and its backward) as one fused HIP
    row kernel each way -- the whole-sequence attention kernels never materialise P."""
    B, S, three_d = qkv.shape
    D = three_d // 3
    hd = D // heads
    q, k, v = qkv.view(B, S, 3, heads, hd).unbind(2)
    z = torch.einsum("bqhd,bkhd->bhqk", q.float() / math.sqrt(hd), k.float())
    p = Dr.softmax_dropout(z, rate, rng, seed)
    return torch.einsum("bhqk,bkhd->bqhd", p, v.float()).reshape(B, S, D).to(qkv.dtype)


def droppath_mask(rate: float, batch: int, rng, device, det: bool):
    """Per-sample keep mask / keep_prob (Flax Dropout with broadcast_dims), or None."""
    if rate <= 0.0 or det:
        return None
    keep = 1.0 - rate
    m = (torch.rand((batch,), generator=rng, device=device) < keep).float() / keep
    return m


def droppath_masks(layers, batch: int, rng, device, det: bool):
    """Every droppath mask of a layer stack in one draw (three kernels instead of three or four
    per mask: 36 masks per ViT-B finetune step), sliced per layer in draw order; None entries
    for layers without droppath.  Also what activation checkpointing hands to the recompute."""
    counts = [(layer.droppath_rate, layer.n_droppath) for layer in layers]
    total = sum(n for r, n in counts if r > 0.0)
    if det or total == 0:
        return [None] * len(layers)
    u = torch.rand((total, batch), generator=rng, device=device)
    # runs of equal rate get one select each (Python-scalar keep: no host->device copy, so
    # the draw is legal inside a captured graph); a uniform rate is a single kernel
    runs, i = [], 0
    for r, n in counts:
        if r > 0.0:
            if runs and runs[-1][0] == r:
                runs[-1][2] += n
            else:
                runs.append([r, i, n])
            i += n
    parts = [torch.where(u[a:a + n] < 1.0 - r, 1.0 / (1.0 - r), 0.0) for r, a, n in runs]
    pool = parts[0] if len(parts) == 1 else torch.cat(parts)
    out, i = [], 0
    for r, n in counts:
        if r > 0.0:
            out.append(pool[i:i + n])
            i += n
        else:
            out.append(None)
    return out


def dropout_seed_pool(layers, rng, device, det: bool, head=None):
    """Every dropout seed of a layer stack from one draw (one kernel per step instead of one per
    layer), sliced per layer in _layer_seeds order; None entries for layers without dropout.  The
    activation-checkpoint recompute gets the same slices.  ``head`` = (x, rate): the stack's input
    dropout takes the pool's first seed and is applied here (returned as the first element)."""
    use = [(not det) and 0.0 < getattr(layer, "dropout_rate", 0.0) < 1.0 for layer in layers]
    hd = head is not None and not det and 0.0 < head[1] < 1.0
    total = sum(layer.n_seeds for layer, u in zip(layers, use) if u) + int(hd)
    x = head[0] if head is not None else None
    if head is not None and not hd:
        x = _dropout(x, head[1], rng, det)  # rate 0 / det: identity; rate >= 1: zeros
    if total == 0:
        return x, [None] * len(layers)
    pool = Dr.draw_seeds(rng, device, total)
    if hd:
        x = Dr.dropout(x, head[1], rng, pool[0])
    out, i = [], int(hd)
    for layer, u in zip(layers, use):
        if u:
            out.append(pool[i:i + layer.n_seeds])
            i += layer.n_seeds
        else:
            out.append(None)
    return x, out


def _mask(masks, k, rate, batch, rng, device, det):
    """k-th pooled mask of a layer, or a fresh draw when the layer was called without a pool."""
    if masks is not None:
        return masks[k]
    return droppath_mask(rate, batch, rng, device, det)


# ---------------------------------------------------------------------------------- blocks
class JumboLayer:
    """Encoder block (modeling.py:169-206)."""

    def __init__(self, store, path, cfg: ViTConfig, jumbo_mlp: FeedForward, trainable=True):
        D, J = cfg.dim, cfg.jumbo_dim
        self.cfg = cfg
        self.C = cfg.num_cls_tokens
        self.attn = Attention(store, path + ("attn",), D, cfg.heads, cfg.dropout, trainable)
        self.ff = FeedForward(store, path + ("ff",), D, cfg.hidden_dim, cfg.dropout, trainable)
        self.norm1 = LayerNorm(store, path + ("norm1",), D, trainable)
        self.norm2 = LayerNorm(store, path + ("norm2",), D, trainable)
        self.norm3 = LayerNorm(store, path + ("norm3",), J, trainable)
        self.jumbo_mlp = jumbo_mlp
        self.scale1 = self.scale2 = self.scale3 = None
        if cfg.layerscale:
            self.scale1 = store.handle(store.add(path + ("scale1",), (D,), const_(1e-4), trainable=trainable))
            self.scale2 = store.handle(store.add(path + ("scale2",), (D,), const_(1e-4), trainable=trainable))
            self.scale3 = store.handle(store.add(path + ("scale3",), (J,), const_(1e-4), trainable=trainable))

    n_droppath = 3  # masks per call, draw order: attention, jumbo, patch FF residual
    n_seeds = 6  # dropout seeds per call (_layer_seeds order)

    @property
    def droppath_rate(self):
        return self.cfg.droppath

    @property
    def dropout_rate(self):
        return self.cfg.dropout

    def __call__(self, x, rng=None, det=True, link_in=None, link_out=None, masks=None, seeds=None):
        B, S, D = x.shape
        C = self.C
        p = self.cfg.droppath
        sd = seeds if seeds is not None else _layer_seeds(self.cfg.dropout, rng, x.device, det, 6)
        if use_fused_blocks() and self.cfg.dropout < 1.0:
            m1 = _mask(masks, 0, p, B, rng, x.device, det)
            m3 = _mask(masks, 1, p, B, rng, x.device, det)
            m2 = _mask(masks, 2, p, B, rng, x.device, det)
            return blocks.jumbo_block(self, x, m1, m2, m3, link_in, link_out, _drops(sd, self.cfg.dropout, True))
        h = self.norm1(x)
        a = self.attn(h, B, S, rng, det, sd and sd[0:2])
        x = Fn.residual(x, a, self.scale1, _mask(masks, 0, p, B, rng, x.device, det))

        # NB: the jumbo residual is added to the *normalized* CLS token (modeling.py:197-199),
        # so the CLS stream is re-normalized by norm3 in every layer.
        cls = x[:, :C].reshape(B, 1, C * D)
        hc = self.norm3(cls, out_dtype=torch.float32)  # [B, J] fp32 residual base
        yc = self.jumbo_mlp(hc.to(self.norm3.g.store.compute_dtype), rng, det, sd and sd[2:4])
        xc = Fn.residual(hc.view(B, 1, C * D), yc, self.scale3, _mask(masks, 1, p, B, rng, x.device, det))

        pt = x[:, C:]
        hp = self.norm2(pt)
        yp = self.ff(hp, rng, det, sd and sd[4:6])
        xp = Fn.residual(pt, yp, self.scale2, _mask(masks, 2, p, B, rng, x.device, det))
        return torch.cat([xc.view(B, C, D), xp], 1)


class ViTLayer:
    """Standard pre-LN block used by the MAE decoder (modeling.py:150-167)."""

    def __init__(self, store, path, dim, heads, layerscale, dropout, droppath, trainable=True):
        self.attn = Attention(store, path + ("attn",), dim, heads, dropout, trainable)
        self.ff = FeedForward(store, path + ("ff",), dim, 4 * dim, dropout, trainable)
        self.norm1 = LayerNorm(store, path + ("norm1",), dim, trainable)
        self.norm2 = LayerNorm(store, path + ("norm2",), dim, trainable)
        self.droppath = droppath
        self.scale1 = self.scale2 = None
        if layerscale:
            self.scale1 = store.handle(store.add(path + ("scale1",), (dim,), const_(1e-4), trainable=trainable))
            self.scale2 = store.handle(store.add(path + ("scale2",), (dim,), const_(1e-4), trainable=trainable))

    n_droppath = 2  # masks per call, draw order: attention, FF residual
    n_seeds = 4  # dropout seeds per call (_layer_seeds order)

    @property
    def droppath_rate(self):
        return self.droppath

    @property
    def dropout_rate(self):
        return self.attn.dropout

    def __call__(self, x, rng=None, det=True, link_in=None, link_out=None, masks=None, seeds=None):
        B, S, D = x.shape
        p = self.droppath
        sd = seeds if seeds is not None else _layer_seeds(self.attn.dropout, rng, x.device, det, 4)
        if use_fused_blocks() and self.attn.dropout < 1.0:
            m1 = _mask(masks, 0, p, B, rng, x.device, det)
            m2 = _mask(masks, 1, p, B, rng, x.device, det)
            return blocks.vit_block(self, x, m1, m2, link_in, link_out, _drops(sd, self.attn.dropout, False))
        h = self.norm1(x)
        a = self.attn(h, B, S, rng, det, sd and sd[0:2])
        x = Fn.residual(x, a, self.scale1, _mask(masks, 0, p, B, rng, x.device, det))
        h = self.norm2(x)
        f = self.ff(h, rng, det, sd and sd[2:4])
        return Fn.residual(x, f, self.scale2, _mask(masks, 1, p, B, rng, x.device, det))


# ------------------------------------------------------------------------------ encoder
class JumboViT:
    """Jumbo ViT encoder (modeling.py:221-274).  Segments are allocated so that the flat
    buffer order is the reverse of backward readiness (good all-reduce buckets)."""

    def __init__(self, store: ParamStore, cfg: ViTConfig, prefix=("model",), trainable=True):
        self.cfg = cfg
        D, p, g = cfg.dim, cfg.patch_size, cfg.grid
        P = prefix
        # embed/wte: HWIO (p,p,3,D) == GEMM kernel [(ph,pw,c), D], stored D x (p*p*3)
        self.wte_k = store.handle(_dense_kernel(store, P + ("embed", "wte", "kernel"), (p, p, 3), (D,), trainable))
        self.wte_b = store.handle(_bias(store, P + ("embed", "wte", "bias"), (D,), trainable))
        self.wpe = None
        if cfg.posemb == "learnable":
            self.wpe = store.handle(store.add(P + ("embed", "wpe"), (g * g, D), trunc_normal_,
                                              flax_shape=(g, g, D),
                                              to_flax=lambda a, s=(g, g, D): a.reshape(s),
                                              from_flax=lambda a, n=g * g, d=D: a.reshape(n, d),
                                              trainable=trainable))
        self.cls_tokens = store.handle(store.add(P + ("cls_tokens",), (1, cfg.num_cls_tokens, D), zeros_,
                                                 trainable=trainable))
        self.jumbo_mlp = FeedForward(store, P + ("jumbo_mlp",), cfg.jumbo_dim, 4 * cfg.jumbo_dim,
                                     cfg.dropout, trainable)
        # shared by every layer: its weight gradients are batched into one GEMM over all layers'
        # rows at the end of backward (ops/prims.py linear_bwd / flush_deferred_wgrads)
        self.jumbo_mlp.w1.k.defer_wgrad = True
        self.jumbo_mlp.w2.k.defer_wgrad = True
        store.pad()
        self.layers = []
        for i in range(cfg.layers):
            self.layers.append(JumboLayer(store, P + (f"layer_{i}",), cfg, self.jumbo_mlp, trainable))
            store.pad()
        self.norm = LayerNorm(store, P + ("norm",), D, trainable)
        store.pad()
        self._posemb_cache = {}

    def posemb_table(self, device) -> torch.Tensor | None:
        """Constant sincos table [g*g, D] (fp32), or None for learnable posemb."""
        if self.cfg.posemb != "sincos2d":
            return None
        key = str(device)
        if key not in self._posemb_cache:
            g = self.cfg.grid
            self._posemb_cache[key] = fixed_sincos2d_embeddings(g, g, self.cfg.dim, device).reshape(g * g, -1)
        return self._posemb_cache[key]

    def embed(self, patches: torch.Tensor, ids: torch.Tensor | None) -> torch.Tensor:
        """patches: [B, n, p*p*3] normalized pixels (already gathered at ``ids`` when given).
        Returns [B, C + n, D] fp32 residual stream."""
        B, n, K = patches.shape
        dt = self.wte_k.store.compute_dtype
        return self.embed_rows(patches.reshape(B * n, K).to(dt), ids, B)

    def embed_rows(self, rows: torch.Tensor, ids: torch.Tensor | None, B: int) -> torch.Tensor:
        """rows: [B*n, p*p*3] patch pixels in the compute dtype (patch ``ids[.., j]`` of each image;
        all patches in order when ``ids`` is None).  Patch-embed GEMM (bias fused), then one
        kernel adds the posemb and writes the CLS + patch rows of the fp32 stream."""
        e = Fn.linear(rows, self.wte_k, self.wte_b)
        if ids is None:
            ids = self._arange(rows.shape[0] // B, rows.device)
        return mae_ops.embed_finish(e, self.cls_tokens, self.wpe, self.posemb_table(rows.device), ids, B)

    def _arange(self, n, device):
        key = ("arange", n, str(device))
        if key not in self._posemb_cache:
            self._posemb_cache[key] = torch.arange(n, device=device)
        return self._posemb_cache[key]

    def blocks(self, x: torch.Tensor, rng=None, det=True) -> torch.Tensor:
        return _run_layers(self.layers, x, rng, det, self.cfg.grad_ckpt, in_dropout=self.cfg.dropout)


def _run_layers(layers, x, rng, det, grad_ckpt, in_dropout=0.0):
    """The layer loop; consecutive fused blocks are chained by ``blocks.Link`` hand-offs (not
    under activation checkpointing, whose recompute would re-run forwards out of order).
    ``in_dropout``: dropout of the stack's input (its seed drawn with the layers' seeds)."""
    masks = droppath_masks(layers, x.shape[0], rng, x.device, det)
    x, seeds = dropout_seed_pool(layers, rng, x.device, det, head=(x, in_dropout))
    if grad_ckpt and torch.is_grad_enabled():
        for layer, m, sd in zip(layers, masks, seeds):
            x = _checkpointed(layer, x, rng, det, m, sd)
        return x
    link = None
    for i, layer in enumerate(layers):
        nxt = None
        if blocks.LINKS and torch.is_grad_enabled():
            up = layers[i + 1] if i + 1 < len(layers) else None
            # the upper block's LN1 rides on this block's last residual pass (forward hand-off)
            ln1 = (up.norm1.g, up.norm1.b) if up is not None and blocks.FWD_LINKS else None
            nxt = blocks.Link(ln1)
        x = layer(x, rng, det, link_in=link, link_out=nxt, masks=masks[i], seeds=seeds[i])
        link = nxt
    return x


def _checkpointed(layer, x, rng, det, masks=None, seeds=None):
    """One layer under activation checkpointing (reference ``nn.remat``, modeling.py:232,280).

    The recompute in backward must see exactly the forward's random draws: droppath / dropout
    masks come from the explicit ``rng`` generator, which ``torch.utils.checkpoint`` does not
    restore.  So the generator state at the layer's entry is snapshotted; the first call runs on
    the shared generator (advancing it as an un-checkpointed run would) and the recompute runs on
    a private generator restored to the snapshot.  The recompute also re-records no parameter
    uses: the data-parallel reducer expects one ``ready`` per FORWARD use, and backward runs once.
    """
    store = layer.norm1.g.store
    state = rng.get_state() if rng is not None else None
    calls = [0]

    def run(inp):
        calls[0] += 1
        if calls[0] == 1:
            return layer(inp, rng, det, masks=masks, seeds=seeds)
        g = None
        if rng is not None:
            g = torch.Generator(device=rng.device)
            g.set_state(state)
        with store.uses_suppressed():
            return layer(inp, g, det, masks=masks, seeds=seeds)

    return torch.utils.checkpoint.checkpoint(run, x, use_reentrant=False)


class MAEDecoder:
    """MAE decoder (modeling.py:276-298); fixed sincos posemb on patch tokens only."""

    def __init__(self, store: ParamStore, cfg: DecoderConfig, prefix=("decoder_model",)):
        self.cfg = cfg
        self.layers = []
        for i in range(cfg.dec_layers):
            self.layers.append(ViTLayer(store, prefix + (f"dec_layer_{i}",), cfg.dec_dim, cfg.dec_heads,
                                        cfg.dec_layerscale, cfg.dec_dropout, cfg.dec_droppath))
            store.pad()
        self.dec_norm = LayerNorm(store, prefix + ("dec_norm",), cfg.dec_dim)
        store.pad()
        self._posemb_cache = {}

    def posemb_table(self, device) -> torch.Tensor:
        key = str(device)
        if key not in self._posemb_cache:
            g = self.cfg.grid
            self._posemb_cache[key] = fixed_sincos2d_embeddings(g, g, self.cfg.dec_dim, device).reshape(g * g, -1)
        return self._posemb_cache[key]

    def blocks(self, x, rng=None, det=True):
        return _run_layers(self.layers, x, rng, det, self.cfg.grad_ckpt)


# --------------------------------------------------------------------------------- heads
class LinearCLS:
    """[SyncBatchNorm] -> Dense(labels) on the 3*D jumbo token (modeling.py:209-219)."""

    def __init__(self, store: ParamStore, path, dim: int, labels: int, batch_norm: bool):
        self.batch_norm = batch_norm
        self.bn_scale = self.bn_bias = None
        if batch_norm:
            self.bn_scale = store.handle(store.add(path + ("BatchNorm_0", "scale"), (dim,), ones_))
            self.bn_bias = store.handle(store.add(path + ("BatchNorm_0", "bias"), (dim,), zeros_))
        self.dense = Dense(store, path + ("Dense_0",), dim, labels)
        store.pad()
        self.dim = dim
        # Flax BatchNorm running statistics (collection "batch_stats")
        self.running_mean: torch.Tensor | None = None
        self.running_var: torch.Tensor | None = None

    def init_stats(self, device):
        if self.batch_norm:
            self.running_mean = torch.zeros(self.dim, device=device)
            self.running_var = torch.ones(self.dim, device=device)

    def __call__(self, x: torch.Tensor, det: bool, group=None) -> torch.Tensor:
        if self.batch_norm:
            from ..parallel.syncbn import sync_batch_norm
            x = sync_batch_norm(x, self.bn_scale, self.bn_bias, self.running_mean, self.running_var,
                                training=not det, momentum=0.99, eps=1e-5, group=group)
        dt = self.dense.k.store.compute_dtype
        return self.dense(x.to(dt)).float()
