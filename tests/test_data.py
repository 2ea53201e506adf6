"""Shard reading, transforms, augmentation grammar, collates, loaders."""

import io
import tarfile

import numpy as np
import pytest
import torch
from PIL import Image

from jumbo_mae_tpu_amd.data import shards as S
from jumbo_mae_tpu_amd.data.autoaugment import augmix_transform, auto_augment_transform, rand_augment_transform
from jumbo_mae_tpu_amd.data.loader import ShardDataset, collate_and_pad, collate_and_shuffle, repeat_samples
from jumbo_mae_tpu_amd.data.transforms import RandomResizedCrop, Resize, create_transforms


def _make_tar(path, n, start=0, size=(40, 30)):
    with tarfile.open(path, "w") as tf:
        for i in range(start, start + n):
            img = Image.fromarray(np.full((size[1], size[0], 3), i % 255, np.uint8))
            buf = io.BytesIO()
            img.save(buf, format="JPEG")
            for ext, data in (("jpg", buf.getvalue()), ("cls", str(i % 7).encode())):
                ti = tarfile.TarInfo(f"sample{i:05d}.{ext}")
                ti.size = len(data)
                tf.addfile(ti, io.BytesIO(data))


def test_brace_expand():
    assert S.brace_expand("a-{000..002}.tar") == ["a-000.tar", "a-001.tar", "a-002.tar"]
    assert S.brace_expand("x{a,b}y{1..2}") == ["xay1", "xay2", "xby1", "xby2"]
    assert len(S.shard_list("t-{0000..1023}.tar")) == 1024


def test_tar_samples_grouping(tmp_path):
    p = str(tmp_path / "s-0.tar")
    _make_tar(p, 5)
    samples = list(S.tar_samples(p))
    assert len(samples) == 5
    assert set(samples[0]) >= {"__key__", "jpg", "cls"}
    assert S.decode_cls(samples[3]["cls"]) == 3
    assert S.decode_pil(samples[0]["jpg"]).size == (40, 30)


def test_detshuffle_deterministic():
    a = list(S.detshuffle(range(100), 10, seed=3))
    b = list(S.detshuffle(range(100), 10, seed=3))
    assert a == b and sorted(a) == list(range(100)) and a != list(range(100))


def test_transforms_shapes():
    img = Image.fromarray(np.random.randint(0, 255, (300, 400, 3), np.uint8))
    for crop in ("rrc", "src", "none"):
        tr, va = create_transforms(crop, 64, "rand-m9-mstd0.5-inc1", 0.3, 0.25, 0.875)
        out = tr(img)
        assert out.shape == (3, 64, 64) and out.dtype == np.uint8
        assert va(img).shape == (3, 64, 64)
    assert Resize(73)(img).size == (97, 73)
    i, j, h, w = RandomResizedCrop(64, scale=(0.2, 1.0)).get_params(400, 300)
    assert 0 <= i and 0 <= j and i + h <= 300 and j + w <= 400


@pytest.mark.parametrize("spec", ["rand-m9-mstd0.5-inc1", "rand-m7-n3-p1.0", "augmix-m3-w3-d-1", "original"])
def test_augment_grammar(spec):
    img = Image.fromarray(np.random.randint(0, 255, (64, 64, 3), np.uint8))
    hp = {"translate_const": 28, "img_mean": (124, 116, 104)}
    if spec.startswith("rand"):
        t = rand_augment_transform(spec, hp)
    elif spec.startswith("augmix"):
        t = augmix_transform(spec, dict(hp, translate_pct=0.3))
    else:
        t = auto_augment_transform(spec, hp)
    for _ in range(5):
        out = t(img)
        assert out.size == (64, 64)
    if spec == "rand-m7-n3-p1.0":
        assert t.n == 3 and t.ops[0].prob == 1.0 and t.ops[0].magnitude == 7


def test_collates():
    batch = [np.full((3, 2, 2), i, np.uint8) for i in range(6)]
    out = collate_and_shuffle(batch, repeats=3)
    assert [int(x[0, 0, 0]) for x in out] == [0, 3, 1, 4, 2, 5]
    lab = [(np.zeros((3, 2, 2), np.uint8), 5)] * 3
    imgs, labels = collate_and_pad(lab, batch_size=5)
    assert imgs.shape == (5, 3, 2, 2) and labels.tolist() == [5, 5, 5, -1, -1]
    assert int(imgs[4].max()) == 255  # uint8 -1 == 255 like the reference's full_like(-1)
    assert len(list(repeat_samples([1, 2], 3))) == 6


def test_shard_dataset_rank_split(tmp_path):
    for k in range(4):
        _make_tar(str(tmp_path / f"s-{k}.tar"), 6, start=k * 6)
    spec = str(tmp_path / "s-{0..3}.tar")
    tr, va = create_transforms("none", 16, "none", 0.0, 0.0, 1.0)
    seen = []
    for rank in range(2):
        ds = ShardDataset(spec, "finetune", va, train=False, rank=rank, world=2, image_size=16)
        items = list(ds)
        assert len(items) == 12
        seen += [int(x[0][0, 0, 0]) for x in items]
    assert len(seen) == 24
    ds = ShardDataset(spec, "pretrain", tr, train=True, repeats=2, rank=0, world=1, image_size=16)
    it = iter(ds)
    first = [next(it) for _ in range(4)]
    assert first[0].shape == (3, 16, 16)


def test_loader_synthetic_workers():
    from types import SimpleNamespace

    from jumbo_mae_tpu_amd.data.loader import create_dataloaders
    args = SimpleNamespace(random_crop="rrc", image_size=32, auto_augment="none", color_jitter=0.0,
                           random_erasing=0.0, test_crop_ratio=0.875, train_dataset_shards="synthetic:64:10",
                           valid_dataset_shards="synthetic:10:10", mode="finetune", augment_repeats=1,
                           shuffle_seed=0, train_batch_size=8, grad_accum=1, train_loader_workers=2,
                           valid_batch_size=4, valid_loader_workers=1)
    tl, vl = create_dataloaders(args)
    x, y = next(iter(tl))
    assert x.shape == (8, 3, 32, 32) and x.dtype == torch.uint8 and y.shape == (8,)
    batches = list(vl)
    assert sum(int((b[1] != -1).sum()) for b in batches) == 10
