"""Training / validation data loaders.

Reference ``create_dataloaders`` (/root/reference/src/dataset.py:100-161) with helpers
``repeat_samples`` / ``collate_and_shuffle`` / ``collate_and_pad`` (:85-97).
* train: infinite cycle over deterministically shuffled shards, split by rank then by worker,
  sample shuffle buffer, decode, repeated augmentation (``augment_repeats`` deep copies, and the
  collate re-orders the batch as batch[0::r] + batch[1::r] + ... so the copies of one image land
  far apart), per-rank batch = train_batch_size // world_size // grad_accum, drop_last.
* valid: one pass, rank split, last batch padded with ``-1`` (uint8 images become 255, labels -1).
* ``synthetic:N[:C]`` shard spec: N random images with C classes (plumbing tests / benchmarks;
  no dataset is reachable offline).
* Device augment (``--device-augment``, on by default on a GPU when the train transform is the
  pretraining one -- RandomResizedCrop + flip, nothing else): the workers decode, draw the crop /
  flip parameters from the same per-sample RNG as the PIL path and ship only the crop window plus
  a descriptor (``DeviceRRCParams``, packed per batch by ``collate_packed``); the resize and flip
  run on the GPU (csrc/augment.hip), bit-exact to PIL's bicubic, when ``DevicePrefetcher`` lands
  the batch.  A worker then spends its time on the JPEG decode only (profiles/r5_data_rate.txt).
Per-rank split replaces the reference's per-host split (one process per GPU here).
"""

from __future__ import annotations

import copy
import itertools
import math
import random
from functools import partial
from typing import NamedTuple

import numpy as np
import torch
from torch.utils.data import DataLoader, IterableDataset, get_worker_info

from . import shards as S
from .transforms import RandomResizedCrop, create_transforms

RRC_TAB = 13  # csrc/augment.hip descriptor width
RRC_KMAX = 24  # csrc/augment.hip taps per output pixel


class PackedImages(NamedTuple):
    """A batch for the device augment: concatenated HWC uint8 crop windows + [B, 13] descriptors
    (csrc/augment.hip), the scratch size of the horizontal pass and the output size."""
    src: torch.Tensor
    tab: torch.Tensor
    tmp_bytes: int
    rows_max: int
    size: int


def _span(n: int, a: int, c: int, out: int) -> tuple[int, int]:
    """Input index range a superset of what Pillow's bicubic resample of [a, a + c) -> ``out`` reads."""
    support = 2.0 * max(c / out, 1.0)
    return max(0, math.floor(a - support) - 1), min(n, math.ceil(a + c + support) + 1)


def _taps(c: int, out: int) -> int:
    return math.ceil(2.0 * max(c / out, 1.0)) * 2 + 1  # Pillow's ksize


class DeviceRRCParams:
    """Worker side of the device augment, in place of RandomResizedCrop(scale 0.2-1, bicubic) +
    RandomHorizontalFlip + PILToArray: the same RNG draws in the same order; returns the crop
    window (HWC uint8) and its descriptor.  A crop too large for the kernel's tap budget is resized
    here with PIL and shipped as an identity window."""

    def __init__(self, size: int):
        self.size = size
        self.rrc = RandomResizedCrop(size, scale=(0.2, 1.0))

    def __call__(self, img):
        from PIL import Image
        if img.mode != "RGB":
            img = img.convert("RGB")
        W, H = img.size
        i, j, ch, cw = self.rrc.get_params(W, H)
        flip = int(random.random() < 0.5)
        S = self.size
        if max(_taps(ch, S), _taps(cw, S)) > RRC_KMAX:
            arr = np.asarray(img.resize((S, S), Image.BICUBIC, box=(j, i, j + cw, i + ch)))
            H = W = S
            i = j = 0
            ch = cw = S
        else:
            arr = np.asarray(img)
        y0, y1 = _span(H, i, ch, S)
        x0, x1 = _span(W, j, cw, S)
        win = np.ascontiguousarray(arr[y0:y1, x0:x1])
        return win, np.array([0, y1 - y0, x1 - x0, y0, x0, H, W, i, j, ch, cw, flip, 0], dtype=np.int64)


def collate_packed(batch, repeats: int = 1, size: int = 224):
    """Device-augment collate: the repeat re-ordering of ``collate_and_shuffle``, then windows
    concatenated into one flat buffer with offsets written into the descriptors."""
    batch = sum([batch[i::repeats] for i in range(repeats)], [])
    labels = None
    if isinstance(batch[0][0], tuple):  # ((win, desc), label)
        labels = torch.tensor([b[1] for b in batch])
        batch = [b[0] for b in batch]
    tab = np.stack([d for _, d in batch])
    sizes = np.array([w.size for w, _ in batch], dtype=np.int64)
    tab[:, 0] = np.concatenate([[0], np.cumsum(sizes)[:-1]])
    rows = tab[:, 1]
    tab[:, 12] = np.concatenate([[0], np.cumsum(rows * size * 3)[:-1]])
    src = torch.from_numpy(np.concatenate([w.reshape(-1) for w, _ in batch]))
    packed = PackedImages(src, torch.from_numpy(tab), int((rows * size * 3).sum()), int(rows.max()), size)
    return packed if labels is None else (packed, labels)


def unpack_on_device(p: PackedImages, device) -> torch.Tensor:
    """uint8 [B, 3, S, S] from a packed batch: H2D of the windows, then the resize / flip kernels."""
    from ..ops import _ext
    src = p.src.to(device, non_blocking=True)
    tab = p.tab.to(device, non_blocking=True)
    return _ext.load(True).rrc_resize(src, tab, p.size, p.tmp_bytes, p.rows_max)


def device_augment_ok(args) -> bool:
    """The train transform is RandomResizedCrop + flip only (the pretraining presets)."""
    return (getattr(args, "random_crop", "rrc") == "rrc" and getattr(args, "auto_augment", "none") in ("none", "", None)
            and not getattr(args, "color_jitter", 0.0) and not getattr(args, "random_erasing", 0.0))


def repeat_samples(samples, repeats: int = 1):
    for s in samples:
        for _ in range(repeats):
            yield copy.deepcopy(s)


def _stack(items):
    first = items[0]
    if isinstance(first, tuple):
        return tuple(_stack([it[i] for it in items]) for i in range(len(first)))
    if isinstance(first, np.ndarray):
        return torch.from_numpy(np.stack(items))
    if isinstance(first, torch.Tensor):
        return torch.stack(items)
    return torch.tensor(items)


def collate_and_shuffle(batch, repeats: int = 1):
    return _stack(sum([batch[i::repeats] for i in range(repeats)], []))


def _minus_one_like(x):
    if isinstance(x, np.ndarray):
        # torch.full_like(uint8, -1) wraps to 255 in the reference; numpy 2 refuses -1 for uint8
        return np.full_like(x, np.iinfo(x.dtype).max if x.dtype.kind == "u" else -1)
    return -1


def collate_and_pad(batch, batch_size: int = 1):
    first = batch[0]
    if isinstance(first, tuple):
        pad = tuple(_minus_one_like(x) for x in first)
    else:
        pad = _minus_one_like(first)
    return _stack(list(batch) + [pad] * (batch_size - len(batch)))


def sample_seed(seed: int, rank: int, wid: int, index: int) -> int:
    """Seed of the augmentation draws of one training sample: sample ``index`` of worker ``wid``'s
    post-repeat stream on ``rank``.  Seeding per sample (not once per worker) makes a sample's
    augmentation independent of how many samples came before it, so a resumed run that skips the
    consumed samples without decoding them reproduces the uninterrupted stream exactly."""
    h = (seed * 1_000_003 + rank * 92_821 + wid * 7_919) & 0xFFFFFFFF
    return (h * 2_654_435_761 + index * 40_503 + 0x9E3779B9) % (2 ** 32)


def worker_skip(batches: int, wid: int, nw: int) -> int:
    """Batches that worker ``wid`` of ``nw`` delivered among the first ``batches`` of a DataLoader
    (the loader takes batches from its workers round-robin)."""
    return (batches - wid + nw - 1) // nw if batches > wid else 0


class ShardDataset(IterableDataset):
    def __init__(self, spec, mode: str, transform, train: bool, repeats: int = 1, seed: int = 0,
                 rank: int = 0, world: int = 1, shuffle_buffer: int = 2000, image_size: int = 224,
                 skip_batches: int = 0, batch_size: int = 1):
        self.spec, self.mode, self.transform, self.train = spec, mode, transform, train
        self.repeats, self.seed, self.rank, self.world = repeats, seed, rank, world
        self.shuffle_buffer = shuffle_buffer
        self.image_size = image_size
        # resume: the first ``skip_batches`` DataLoader batches (of ``batch_size``) were consumed by
        # the interrupted run; each worker skips its share of them without decoding
        self.skip_batches, self.batch_size = skip_batches, batch_size
        # validation batches always carry a label so that padded rows (-1) can be masked out
        self.with_label = mode in ("finetune", "linear") or not train
        self.synthetic = isinstance(spec, str) and spec.startswith("synthetic:")
        self.urls = [] if self.synthetic else S.shard_list(spec)

    # raw (undecoded) records of this rank/worker, one epoch
    def _records(self, epoch: int, wid: int, nw: int):
        if self.synthetic:
            parts = self.spec.split(":")
            n = int(parts[1])
            idx = itertools.islice(range(n), self.rank * nw + wid, None, self.world * nw)
            for i in idx:
                yield {"synthetic": i + (epoch * 7919 if self.train else 0)}
            return
        urls = S.epoch_shards(self.urls, self.seed, epoch, shuffle=self.train)
        total = self.world * nw
        if len(urls) >= total:
            mine = S.split(S.split(urls, self.rank, self.world), wid, nw)
            sample_filter = None
        else:  # fewer shards than consumers: split samples instead of shards
            mine = urls
            sample_filter = (self.rank * nw + wid, total)
        handler = S.ignore_and_continue if self.train else None
        # validation shards are cached locally on the first pass (webdataset cached_tarfile_to_samples)
        it = S.iter_samples(mine, handler) if self.train else S.cached_samples(mine, handler)
        if sample_filter is not None:
            it = itertools.islice(it, sample_filter[0], None, sample_filter[1])
        if self.train:
            it = S.detshuffle(it, self.shuffle_buffer, self.seed * 7 + epoch * 131 + self.rank * 17 + wid)
        yield from it

    def _decode(self, rec):
        """Decoded sample dict of a record, or None (train: a corrupt record is skipped)."""
        if "synthetic" in rec:
            parts = self.spec.split(":")
            ncls = int(parts[2]) if len(parts) > 2 else 1000
            rs = np.random.default_rng(rec["synthetic"])
            arr = rs.integers(0, 256, (self.image_size + 32, self.image_size + 32, 3), dtype=np.uint8)
            from PIL import Image
            return {"jpg": Image.fromarray(arr), "cls": int(rs.integers(0, ncls))}
        try:
            out = {"jpg": S.decode_pil(rec["jpg"])}
            if self.with_label:
                out["cls"] = S.decode_cls(rec["cls"]) if "cls" in rec else 0
            return out
        except Exception:
            if not self.train:
                raise
            return None

    # kept for callers of the one-epoch decoded view
    def _raw(self, epoch: int, wid: int, nw: int):
        for rec in self._records(epoch, wid, nw):
            s = self._decode(rec)
            if s is not None:
                yield s

    def __iter__(self):
        info = get_worker_info()
        wid, nw = (info.id, info.num_workers) if info is not None else (0, 1)
        if self.train:
            # a resumed loader's batch j is batch start + j of the interrupted stream, which worker
            # (start + j) % nw produced: worker w takes over the role of worker (w + start) % nw
            wid = (wid + self.skip_batches) % nw
        random.seed(self.seed * 1000 + self.rank * 97 + wid)
        np.random.seed((self.seed * 1000 + self.rank * 97 + wid) % (2 ** 32))
        if not self.train:
            for s in self._raw(0, wid, nw):
                img = self.transform(s["jpg"])
                yield (img, s["cls"]) if self.with_label else img
            return
        r = max(self.repeats, 1)
        skip = worker_skip(self.skip_batches, wid, nw) * self.batch_size  # post-repeat samples
        index = 0  # position in this worker's post-repeat sample stream
        epoch = 0
        while True:
            for rec in self._records(epoch, wid, nw):
                if skip >= r:  # the whole record (all its repeats) was consumed before the resume
                    skip -= r
                    index += r
                    continue
                s = self._decode(rec)
                if s is None:
                    # a record that fails to decode still takes its r positions, so the per-sample
                    # augmentation seeds of everything after it match a resumed run (whose skip
                    # counts records without decoding them).  Exact resume assumes no corrupt
                    # record BEFORE the resume point: the skip (samples consumed / r records) then
                    # lands one record early per corrupt record and repeats its successor's samples.
                    index += r  # as the decoded path: skip + (r - skip) positions
                    skip = 0
                    continue
                first, skip = skip, 0
                index += first
                for k in range(first, r):
                    # repeated augmentation: deep copies of one decoded sample, own draws each
                    seed = sample_seed(self.seed, self.rank, wid, index)
                    random.seed(seed)
                    np.random.seed(seed)
                    img = self.transform(copy.deepcopy(s["jpg"]) if r > 1 else s["jpg"])
                    index += 1
                    yield (img, s["cls"]) if self.with_label else img
            epoch += 1


def create_dataloaders(args, rank: int = 0, world: int = 1, start_batches: int = 0, device_augment: bool = False):
    """Returns (train_loader | None, valid_loader | None) like dataset.py:100-161.  ``start_batches``
    (resume): train batches already consumed on this rank -- the stream continues after them.
    ``device_augment``: train batches are ``PackedImages`` for ``unpack_on_device`` (requires
    ``device_augment_ok(args)``)."""
    train_t, valid_t = create_transforms(args.random_crop, args.image_size, args.auto_augment, args.color_jitter,
                                         args.random_erasing, args.test_crop_ratio)
    if device_augment:
        assert device_augment_ok(args), "device augment covers RandomResizedCrop + flip only"
        train_t = DeviceRRCParams(args.image_size)
    train_dl = valid_dl = None
    pin = torch.cuda.is_available()
    if getattr(args, "train_dataset_shards", None):
        bs = args.train_batch_size // world // args.grad_accum
        ds = ShardDataset(args.train_dataset_shards, args.mode, train_t, True, args.augment_repeats,
                          args.shuffle_seed, rank, world, image_size=args.image_size,
                          skip_batches=start_batches, batch_size=bs)
        nw = args.train_loader_workers
        collate = (partial(collate_packed, repeats=args.augment_repeats, size=args.image_size) if device_augment
                   else partial(collate_and_shuffle, repeats=args.augment_repeats))
        train_dl = DataLoader(ds, batch_size=bs, num_workers=nw, collate_fn=collate,
                              drop_last=True, pin_memory=pin, prefetch_factor=4 if nw > 0 else None,
                              persistent_workers=nw > 0)
    if getattr(args, "valid_dataset_shards", None):
        ds = ShardDataset(args.valid_dataset_shards, args.mode, valid_t, False, 1, 0, rank, world,
                          image_size=args.image_size)
        bs = args.valid_batch_size // world
        nw = args.valid_loader_workers
        valid_dl = DataLoader(ds, batch_size=bs, num_workers=nw, collate_fn=partial(collate_and_pad, batch_size=bs),
                              drop_last=False, pin_memory=pin, prefetch_factor=4 if nw > 0 else None,
                              persistent_workers=nw > 0)
    return train_dl, valid_dl


class SyntheticGPUImages:
    """Infinite GPU-resident random uint8 batches (benchmarks: no host decode / H2D in the loop)."""

    def __init__(self, batch: int, image_size: int, device, labels: int = 0, seed: int = 0, pool: int = 2):
        g = torch.Generator(device=device).manual_seed(seed)
        self.imgs = [torch.randint(0, 256, (batch, 3, image_size, image_size), dtype=torch.uint8, device=device,
                                   generator=g) for _ in range(pool)]
        self.labels = [torch.randint(0, max(labels, 1), (batch,), device=device, generator=g) for _ in range(pool)]
        self.with_labels = labels > 0
        self.i = 0

    def __iter__(self):
        return self

    def __next__(self):
        k = self.i % len(self.imgs)
        self.i += 1
        return (self.imgs[k], self.labels[k]) if self.with_labels else self.imgs[k]
