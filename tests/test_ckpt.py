"""Flax msgpack wire format, converters, pretrained loading, resume sidecar."""

import os

import msgpack
import numpy as np
import pytest
import torch

from jumbo_mae_tpu_amd.ckpt import msgpack_flax as M
from jumbo_mae_tpu_amd.ckpt.checkpoint import (AsyncCheckpointWriter, load_params, load_pretrained_params,
                                               load_resume_state, save_params, save_resume_state, writer)
from jumbo_mae_tpu_amd.ckpt.convert import flax_to_torch, torch_to_flax
from jumbo_mae_tpu_amd.config import DecoderConfig, ViTConfig
from jumbo_mae_tpu_amd.models.classifier import FinetuneModel
from jumbo_mae_tpu_amd.models.mae import PretrainModel


def test_msgpack_wire_format_fixture():
    """Hand-built Flax-style bytes (ExtType 1 = (shape, dtype name, raw C bytes)) decode correctly."""
    arr = np.arange(6, dtype=np.float32).reshape(2, 3)
    payload = msgpack.packb(((2, 3), "float32", arr.tobytes("C")), use_bin_type=True)
    scal = msgpack.packb(((), "int32", np.int32(7).tobytes()), use_bin_type=True)
    blob = msgpack.packb({"model": {"w": msgpack.ExtType(1, payload)}, "n": msgpack.ExtType(3, scal),
                          "c": msgpack.ExtType(2, msgpack.packb((1.0, 2.0)))})
    tree = M.msgpack_restore(blob)
    np.testing.assert_array_equal(tree["model"]["w"], arr)
    assert tree["n"] == 7 and tree["c"] == complex(1, 2)
    # our writer produces the same ext encoding
    ours = msgpack.unpackb(M.msgpack_serialize({"model": {"w": arr}}), raw=False)
    assert ours["model"]["w"].code == 1
    shape, dt, raw = msgpack.unpackb(ours["model"]["w"].data, raw=True)
    assert tuple(shape) == (2, 3) and dt == b"float32" and raw == arr.tobytes()


def test_msgpack_chunked(monkeypatch):
    monkeypatch.setattr(M, "MAX_CHUNK_SIZE", 64)
    a = np.random.randn(10, 7).astype(np.float32)
    data = M.msgpack_serialize({"a": a, "b": {"c": np.ones(3, np.float32)}})
    raw = msgpack.unpackb(data, raw=False, ext_hook=M._ext_unpack)
    assert raw["a"][M.CHUNK_KEY] is True
    back = M.msgpack_restore(data)
    np.testing.assert_array_equal(back["a"], a)


def _pre():
    vc = ViTConfig(layers=2, dim=32, heads=4, labels=0, image_size=32, patch_size=8, posemb="sincos2d",
                   layerscale=True)
    return PretrainModel(vc, DecoderConfig(dec_layers=1, dec_dim=16, dec_heads=2, image_size=32, patch_size=8)).to("cpu")


def test_store_flax_roundtrip(tmp_path):
    m = _pre()
    m.store.master.normal_()
    tree = m.flax_params()
    assert tree["model"]["layer_0"]["attn"]["wq"]["kernel"].shape == (32, 4, 8)
    assert tree["model"]["layer_0"]["attn"]["wo"]["kernel"].shape == (4, 8, 32)
    assert tree["model"]["embed"]["wte"]["kernel"].shape == (8, 8, 3, 32)
    assert tree["model"]["cls_tokens"].shape == (1, 3, 32)
    assert tree["model"]["jumbo_mlp"]["w1"]["kernel"].shape == (96, 384)
    assert tree["image_mask_embedding"].shape == (1, 1, 16)
    url = save_params(str(tmp_path), "x", tree, "last")
    writer().flush()
    m2 = _pre()
    loaded, total = m2.load_flax_params(load_params(url))
    assert loaded == total
    for s in m.store.segments:  # (padding between segment groups is not part of the tree)
        assert torch.equal(m2.store.master[s.offset:s.offset + s.numel], m.store.master[s.offset:s.offset + s.numel])


def test_converters_roundtrip():
    vc = ViTConfig(layers=2, dim=32, heads=4, labels=10, image_size=32, patch_size=8, posemb="learnable",
                   layerscale=True, image_mask_ratio=None)
    m = FinetuneModel(vc).to("cpu")
    m.store.master.normal_()
    tree = m.flax_params()
    sd = flax_to_torch(tree)
    assert sd["blocks.1.attn.qkv.weight"].shape == (96, 32)
    assert sd["patch_embed.proj.weight"].shape == (32, 3, 8, 8)
    assert sd["pos_embed"].shape == (1, 3 + 16, 32)
    assert "jumbo_mlp.fc2.weight" in sd and "blocks.0.norm3.weight" in sd and "blocks.0.ls3.gamma" in sd
    back = torch_to_flax(sd, num_heads=4)
    fl_a = M.flatten_tree(tree)
    fl_b = M.flatten_tree(back)
    assert set(fl_a) == set(fl_b)
    for k in fl_a:
        np.testing.assert_allclose(fl_a[k], fl_b[k], atol=1e-6, err_msg=str(k))


@pytest.mark.parametrize("image_size", [224, 448])
def test_converter_sincos_grid_follows_image_size(image_size):
    """A sincos model has no wpe leaf: the exported pos_embed grid comes from --image-size."""
    from jumbo_mae_tpu_amd.utils.posemb import _sincos2d_np
    vc = ViTConfig(layers=1, dim=32, heads=4, labels=10, image_size=image_size, patch_size=16, posemb="sincos2d",
                   image_mask_ratio=None)
    m = FinetuneModel(vc).to("cpu")
    tree = m.flax_params()
    sd = flax_to_torch(tree, image_size=image_size)
    g = image_size // 16
    assert sd["pos_embed"].shape == (1, 3 + g * g, 32)
    np.testing.assert_allclose(sd["pos_embed"][0, 3:], _sincos2d_np(g, g, 32).reshape(g * g, 32), atol=1e-6)
    back = torch_to_flax(sd, num_heads=4, learnable_posemb=False)
    fl_a, fl_b = M.flatten_tree(tree), M.flatten_tree(back)
    assert set(fl_a) == set(fl_b)
    for k in fl_a:
        np.testing.assert_allclose(fl_a[k], fl_b[k], atol=1e-6, err_msg=str(k))


def test_load_pretrained_into_finetune(tmp_path):
    pre = _pre()
    pre.store.master.normal_()
    url = save_params(str(tmp_path), "pre", pre.flax_params(), "last")
    writer().flush()
    vc = ViTConfig(layers=2, dim=32, heads=4, labels=10, image_size=32, patch_size=8, posemb="sincos2d",
                   layerscale=True, image_mask_ratio=None)
    ft = FinetuneModel(vc).to("cpu")
    head_before = ft.flax_params()["model"]["head"]["Dense_0"]["kernel"].copy()
    tree = load_pretrained_params(url, ft.flax_params(), log=lambda *a: None)
    ft.store.load_flax_tree(tree, strict=True)
    t = ft.flax_params()["model"]
    p = pre.flax_params()["model"]
    np.testing.assert_array_equal(t["layer_1"]["ff"]["w2"]["kernel"], p["layer_1"]["ff"]["w2"]["kernel"])
    np.testing.assert_array_equal(t["jumbo_mlp"]["w1"]["bias"], p["jumbo_mlp"]["w1"]["bias"])
    np.testing.assert_array_equal(t["head"]["Dense_0"]["kernel"], head_before)


def test_resume_sidecar_and_async_writer(tmp_path):
    w = AsyncCheckpointWriter()
    for i in range(5):
        w.submit(os.path.join(tmp_path, "f.bin"), bytes([i]) * 1000)
    w.flush()
    assert open(os.path.join(tmp_path, "f.bin"), "rb").read() == bytes([4]) * 1000
    assert not [f for f in os.listdir(tmp_path) if ".tmp." in f]
    w.close()
    st = {"step": 3, "optimizer": {"kind": "adamw", "count": 3, "mu": torch.ones(4)}, "rngs": {"noise": torch.ByteTensor(8)}}
    save_resume_state(os.path.join(tmp_path, "s.state.pt"), st)
    writer().flush()
    back = load_resume_state(os.path.join(tmp_path, "s.state.pt"))
    assert back["step"] == 3 and torch.equal(back["optimizer"]["mu"], torch.ones(4))
