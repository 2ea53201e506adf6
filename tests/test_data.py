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


# ---- RandAugment op fixtures: level -> argument values of timm's level mappings, applied through
# PIL directly and compared with our op (sign and resample draws pinned).
def _pinned(monkeypatch, negate):
    import jumbo_mae_tpu_amd.data.autoaugment as A
    monkeypatch.setattr(A.random, "random", lambda: 0.9 if negate else 0.1)
    monkeypatch.setattr(A.random, "choice", lambda seq: seq[0])
    return A


def _img(seed=0, size=(48, 40)):
    return Image.fromarray(np.random.RandomState(seed).randint(0, 256, (size[1], size[0], 3), np.uint8))


@pytest.mark.parametrize("negate", [False, True])
def test_randaugment_geometric_fixtures(monkeypatch, negate):
    from PIL import Image as I
    A = _pinned(monkeypatch, negate)
    img, hp, sgn = _img(), {"translate_const": 100, "img_mean": (1, 2, 3)}, -1 if negate else 1
    bil = I.BILINEAR
    cases = {  # (op, level): expected PIL call; arguments are the timm formula values at level 9
        "Rotate": lambda: img.rotate(27.0 * sgn, resample=bil, fillcolor=(1, 2, 3)),
        "ShearX": lambda: img.transform(img.size, I.AFFINE, (1, 0.27 * sgn, 0, 0, 1, 0), resample=bil,
                                        fillcolor=(1, 2, 3)),
        "ShearY": lambda: img.transform(img.size, I.AFFINE, (1, 0, 0, 0.27 * sgn, 1, 0), resample=bil,
                                        fillcolor=(1, 2, 3)),
        "TranslateX": lambda: img.transform(img.size, I.AFFINE, (1, 0, 90.0 * sgn, 0, 1, 0), resample=bil,
                                            fillcolor=(1, 2, 3)),
        "TranslateYRel": lambda: img.transform(img.size, I.AFFINE, (1, 0, 0, 0, 1, 0.405 * 40 * sgn),
                                               resample=bil, fillcolor=(1, 2, 3)),
    }
    for name, ref in cases.items():
        out = A.NAME_TO_OP[name](img, 9.0, hp)
        assert np.array_equal(np.asarray(out), np.asarray(ref())), name


def test_randaugment_pixel_fixtures(monkeypatch):
    from PIL import ImageEnhance, ImageOps
    A = _pinned(monkeypatch, negate=True)
    img, a = _img(1), np.asarray(_img(1)).astype(np.int32)
    expect = {
        "Posterize": ImageOps.posterize(img, 3), "PosterizeIncreasing": ImageOps.posterize(img, 1),
        "PosterizeOriginal": ImageOps.posterize(img, 7),
        "Solarize": ImageOps.solarize(img, 230), "SolarizeIncreasing": ImageOps.solarize(img, 26),
        "SolarizeAdd": Image.fromarray(np.where(a < 128, np.minimum(a + 99, 255), a).astype(np.uint8)),
        "Color": ImageEnhance.Color(img).enhance(1.72), "Contrast": ImageEnhance.Contrast(img).enhance(1.72),
        "Brightness": ImageEnhance.Brightness(img).enhance(1.72),
        "Sharpness": ImageEnhance.Sharpness(img).enhance(1.72),
        "ColorIncreasing": ImageEnhance.Color(img).enhance(1.0 - 0.81),
        "BrightnessIncreasing": ImageEnhance.Brightness(img).enhance(1.0 - 0.81),
        "AutoContrast": ImageOps.autocontrast(img), "Equalize": ImageOps.equalize(img),
        "Invert": ImageOps.invert(img),
    }
    for name, ref in expect.items():
        out = A.NAME_TO_OP[name](img, 9.0, {})
        assert np.array_equal(np.asarray(out), np.asarray(ref)), name
    # posterize at >= 8 bits is the identity; enhance-increasing is floored at 0.1 beyond level 10
    assert A.NAME_TO_OP["PosterizeOriginal"](img, 10.0, {}) is img
    assert A._enh_inc_level(20.0) == pytest.approx(0.1)


def test_augment_magnitude_noise(monkeypatch):
    from jumbo_mae_tpu_amd.data.autoaugment import AugmentOp
    seen = []
    op = AugmentOp("Rotate", prob=1.0, magnitude=9, hparams={"magnitude_std": 0.5, "magnitude_max": 10})
    op.fn = lambda img, m, hp: seen.append(m) or img
    import random as R
    R.seed(0)
    for _ in range(200):
        op(None)
    assert all(0.0 <= m <= 10.0 for m in seen) and abs(np.mean(seen) - 9.0) < 0.2
    op.mstd = float("inf")  # uniform in [0, m]
    seen.clear()
    for _ in range(200):
        op(None)
    assert 0.0 <= min(seen) and max(seen) <= 9.0 and abs(np.mean(seen) - 4.5) < 0.6


def test_augmix_blended_weights():
    from jumbo_mae_tpu_amd.data.autoaugment import AugMix
    ws, m = np.array([0.2, 0.5, 0.3]), 0.6
    a = AugMix.blended_weights(ws, m)
    # sequential blends img = (1 - a_k) img + a_k chain_k leave weight m*w_k on chain k
    eff, orig = [], 1.0
    for k in range(3):
        eff.append(a[k] * np.prod([1 - a[j] for j in range(k + 1, 3)]))
        orig *= 1 - a[k]
    np.testing.assert_allclose(eff, m * ws, rtol=1e-5)
    assert orig == pytest.approx(1 - m, rel=1e-5)


@pytest.mark.parametrize("spec", ["augmix-m3-w3-d2-b1", "v0", "v0r", "originalr"])
def test_augment_variants_run(spec):
    img = _img(2, (32, 32))
    t = augmix_transform(spec, {}) if spec.startswith("augmix") else auto_augment_transform(spec, {})
    for _ in range(4):
        assert t(img).size == (32, 32)
    if spec == "v0r":
        names = {op.name for sp in t.policy for op in sp}
        assert "PosterizeIncreasing" in names and "Posterize" not in names


def test_random_erasing_fill_matches_uint8_assignment():
    from jumbo_mae_tpu_amd.data.transforms import RandomErasing, erase_fill
    v = np.random.RandomState(0).standard_normal((3, 8, 8)).astype(np.float32)
    t = torch.zeros(3, 8, 8, dtype=torch.uint8)
    t[:] = torch.from_numpy(v)  # what torchvision v2 erase does with value="random"
    assert np.array_equal(erase_fill(v), t.numpy())
    a = np.full((3, 32, 32), 77, np.uint8)
    out = RandomErasing(p=1.0)(a)
    changed = out != 77
    assert changed.any() and set(np.unique(out[changed])) <= set(range(0, 6)) | set(range(250, 256))


# ---- validation shard cache (webdataset cached_tarfile_to_samples)
def test_cached_path_pipe(tmp_path):
    src = tmp_path / "val-0001.tar"
    _make_tar(str(src), 3)
    cache = tmp_path / "cache"
    url = f"pipe:cat {src}"
    p = S.cached_path(url, str(cache))
    assert p.startswith(str(cache)) and p.endswith("val-0001.tar")
    assert open(p, "rb").read() == src.read_bytes()
    src.unlink()  # the second pass reads the cached copy only
    assert S.cached_path(url, str(cache)) == p
    assert [s["__url__"] for s in S.cached_samples([url], directory=str(cache))] == [url] * 3
    assert S.cached_path(str(tmp_path / "x.tar"), str(cache)) == str(tmp_path / "x.tar")  # local: in place


def test_cached_path_failed_pipe(tmp_path):
    cache = tmp_path / "cache"
    with pytest.raises(IOError):
        S.cached_path(f"pipe:cat {tmp_path}/missing.tar", str(cache))
    assert list(cache.iterdir()) == []  # no partial shard left behind
    got = []
    assert list(S.cached_samples([f"pipe:cat {tmp_path}/missing.tar"], handler=got.append,
                                 directory=str(cache))) == []
    assert len(got) == 1


def test_pipe_exit_status_checked(tmp_path):
    src = tmp_path / "s.tar"
    _make_tar(str(src), 2)
    assert len(list(S.tar_samples(f"pipe:cat {src}"))) == 2
    with pytest.raises(IOError):
        list(S.tar_samples(f"pipe:cat {src}; exit 3"))


def test_valid_dataset_uses_cache(tmp_path, monkeypatch):
    for k in range(2):
        _make_tar(str(tmp_path / f"v-{k}.tar"), 4, start=k * 4)
    monkeypatch.setenv("WDS_CACHE", str(tmp_path / "wc"))
    _, va = create_transforms("none", 16, "none", 0.0, 0.0, 1.0)
    spec = f"pipe:cat {tmp_path}/v-{{0..1}}.tar"
    ds = ShardDataset(spec, "finetune", va, train=False, image_size=16)
    assert len(list(ds)) == 8
    assert len(list((tmp_path / "wc").iterdir())) == 2
    assert len(list(ds)) == 8  # second pass from the cache


# ------------------------------------------------------------------ device augment (CPU side)
def _dev_aug_args(spec, workers=0, batch=8):
    from types import SimpleNamespace
    return SimpleNamespace(random_crop="rrc", image_size=224, auto_augment="none", color_jitter=0.0,
                           random_erasing=0.0, test_crop_ratio=0.875, train_dataset_shards=spec,
                           valid_dataset_shards=None, mode="pretrain", train_batch_size=batch, grad_accum=1,
                           augment_repeats=2, shuffle_seed=3, train_loader_workers=workers, valid_batch_size=batch,
                           valid_loader_workers=0)


def test_device_augment_packed_batches_equal_pil(tmp_path):
    """The device-augment workers (decode + the same RNG draws, crop windows + descriptors) and
    the NumPy mirror of csrc/augment.hip reproduce the PIL transform's batches bit for bit,
    repeated augmentation included."""
    from jumbo_mae_tpu_amd.data.jpeg_shards import write_shards
    from jumbo_mae_tpu_amd.data.loader import PackedImages, create_dataloaders
    from jumbo_mae_tpu_amd.data.resample_ref import unpack_packed
    spec = write_shards(str(tmp_path), shards=2, per_shard=12, classes=5, seed=4)
    cpu, _ = create_dataloaders(_dev_aug_args(spec))
    dev, _ = create_dataloaders(_dev_aug_args(spec), device_augment=True)
    for (a, b), _ in zip(zip(cpu, dev), range(3)):
        assert isinstance(b, PackedImages) and b.tab.shape == (8, 13)
        assert b.src.numel() < 8 * 500 * 500 * 3  # crop windows, not whole pictures
        got = unpack_packed(b)
        assert got.shape == tuple(a.shape) and np.array_equal(got, a.numpy())


def test_device_augment_large_crop_fallback():
    """A crop beyond the kernel's tap budget is resized by PIL in the worker and shipped as an
    identity window: same result."""
    import random

    from PIL import Image

    from jumbo_mae_tpu_amd.data.loader import DeviceRRCParams, collate_packed
    from jumbo_mae_tpu_amd.data.resample_ref import unpack_packed
    from jumbo_mae_tpu_amd.data.transforms import create_transforms
    rs = np.random.default_rng(0)
    imgs = [Image.fromarray(rs.integers(0, 256, (h, w, 3), dtype=np.uint8)) for h, w in
            ((1500, 2100), (300, 260), (2600, 1900), (224, 224))]
    cpu_t, _ = create_transforms("rrc", 224, "none", 0.0, 0.0, 0.875)
    dev_t = DeviceRRCParams(224)
    want, got = [], []
    for k, im in enumerate(imgs):
        random.seed(k)
        want.append(cpu_t(im))
        random.seed(k)
        got.append(dev_t(im))
    assert got[0][1][5] == 224  # fell back: identity window
    assert np.array_equal(unpack_packed(collate_packed(got)), np.stack(want))
