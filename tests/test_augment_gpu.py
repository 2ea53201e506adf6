"""Device augment kernels (csrc/augment.hip): RandomResizedCrop (bicubic) + flip on the GPU must be
bit-exact to PIL's transform of the same images with the same RNG draws, through the real loader
(JPEG shards, device-augment workers, packed batches) and the DevicePrefetcher."""

import random

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _args(spec, batch=16):
    from types import SimpleNamespace
    return SimpleNamespace(random_crop="rrc", image_size=224, auto_augment="none", color_jitter=0.0,
                           random_erasing=0.0, test_crop_ratio=0.875, train_dataset_shards=spec,
                           valid_dataset_shards=None, mode="pretrain", train_batch_size=batch, grad_accum=1,
                           augment_repeats=1, shuffle_seed=1, train_loader_workers=2, valid_batch_size=batch,
                           valid_loader_workers=0)


def test_rrc_kernel_matches_pil_through_the_loader(tmp_path):
    from jumbo_mae_tpu_amd.data.jpeg_shards import write_shards
    from jumbo_mae_tpu_amd.data.loader import create_dataloaders
    from jumbo_mae_tpu_amd.train.common import DevicePrefetcher
    spec = write_shards(str(tmp_path), shards=2, per_shard=24, classes=5, seed=9)
    cpu, _ = create_dataloaders(_args(spec))
    dev, _ = create_dataloaders(_args(spec), device_augment=True)
    pf = DevicePrefetcher(dev, torch.device("cuda"))
    n = 0
    for a, b in zip(cpu, pf):
        torch.cuda.synchronize()
        assert b.is_cuda and b.dtype == torch.uint8 and b.shape == a.shape
        assert torch.equal(b.cpu(), a), (b.cpu().int() - a.int()).abs().max()
        n += 1
        if n == 3:
            break
    assert n == 3


@pytest.mark.parametrize("size", [224, 96, 300])
def test_rrc_kernel_matches_pil_random_windows(size):
    """Random pictures, crops (down- and upscaling) and flips; the fallback identity window too."""
    from PIL import Image

    from jumbo_mae_tpu_amd.data.loader import DeviceRRCParams, collate_packed, unpack_on_device
    from jumbo_mae_tpu_amd.data.resample_ref import unpack_packed
    from jumbo_mae_tpu_amd.data.transforms import create_transforms
    rs = np.random.default_rng(size)
    cpu_t, _ = create_transforms("rrc", size, "none", 0.0, 0.0, 0.875)
    dev_t = DeviceRRCParams(size)
    want, got = [], []
    for k in range(24):
        h, w = int(rs.integers(60, 900)), int(rs.integers(60, 900))
        if k == 0:
            h, w = 2400, 1800  # beyond the tap budget at small sizes: PIL in the worker
        im = Image.fromarray(rs.integers(0, 256, (h, w, 3), dtype=np.uint8))
        random.seed(k)
        want.append(cpu_t(im))
        random.seed(k)
        got.append(dev_t(im))
    packed = collate_packed(got, size=size)
    out = unpack_on_device(packed, torch.device("cuda"))
    torch.cuda.synchronize()
    ref = np.stack(want)
    assert np.array_equal(unpack_packed(packed), ref)
    assert np.array_equal(out.cpu().numpy(), ref)
