"""Data parallel ON THE GPU code path (HIP kernels, MFMA GEMMs, deferred jumbo-MLP weight
gradients, bucketed reducer) with two ranks sharing one MI355X through the gloo backend (RCCL
needs one GPU per rank; the 8-GPU RCCL run is the driver's).  DP gradients must equal the
single-process large-batch gradients up to bf16 GEMM rounding."""

import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from jumbo_mae_tpu_amd.config import DecoderConfig, ViTConfig

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cfgs():
    vc = ViTConfig(layers=2, dim=256, heads=4, labels=0, image_size=64, patch_size=8, posemb="sincos2d")
    dc = DecoderConfig(dec_layers=2, dec_dim=256, dec_heads=8, image_size=64, patch_size=8)
    return vc, dc


def _data():
    g = torch.Generator().manual_seed(0)
    imgs = torch.randint(0, 256, (256, 3, 64, 64), dtype=torch.uint8, generator=g)
    noise = torch.rand(64, generator=g)
    return imgs, noise


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from jumbo_mae_tpu_amd.models.mae import PretrainModel
    from jumbo_mae_tpu_amd.parallel.ddp import GradReducer
    vc, dc = _cfgs()
    dev = torch.device("cuda", 0)
    m = PretrainModel(vc, dc).to(dev, torch.bfloat16, seed=rank)
    dist.broadcast(m.store.master, 0)
    m.store.sync_shadow()
    red = GradReducer(m.store, bucket_mb=1.0)
    imgs, noise = _data()
    half = imgs.shape[0] // world
    mine = imgs[rank * half:(rank + 1) * half].to(dev)
    m.store.zero_grad()
    red.begin_step()
    loss = m(mine, noise=noise.to(dev))["loss"]
    loss.backward()
    red.finish()
    torch.cuda.synchronize()
    if rank == 0:
        torch.save({"grad": m.store.grad.cpu(), "master": m.store.master.cpu()}, out)
    dist.barrier()
    dist.destroy_process_group()


def _reference(out):
    torch.cuda.set_device(0)
    from jumbo_mae_tpu_amd.models.mae import PretrainModel
    vc, dc = _cfgs()
    dev = torch.device("cuda", 0)
    m = PretrainModel(vc, dc).to(dev, torch.bfloat16, seed=0)
    imgs, noise = _data()
    a = imgs[:128].to(dev)
    b = imgs[128:].to(dev)
    m.store.zero_grad()
    # same per-rank batches as DP, gradients averaged: exactly the DP computation, no reducer
    (m(a, noise=noise.to(dev))["loss"] * 0.5).backward()
    (m(b, noise=noise.to(dev))["loss"] * 0.5).backward()
    torch.cuda.synchronize()
    torch.save({"grad": m.store.grad.cpu(), "master": m.store.master.cpu()}, out)


def test_dp_two_ranks_on_gpu_match_large_batch():
    port = _free_port()
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "dp.pt")
        ref_out = os.path.join(d, "ref.pt")
        mp.spawn(_worker, args=(2, port, out), nprocs=2, join=True)
        ctx = mp.get_context("spawn")
        p = ctx.Process(target=_reference, args=(ref_out,))
        p.start()
        p.join()
        assert p.exitcode == 0
        r = torch.load(out, weights_only=True)
        ref = torch.load(ref_out, weights_only=True)
    assert torch.equal(r["master"], ref["master"])
    g, gr = r["grad"], ref["grad"]
    assert torch.isfinite(g).all()
    rel = ((g - gr).norm() / gr.norm()).item()
    assert rel < 1e-3, rel
