"""Multi-process data parallel on CPU (gloo, world_size 2): DP gradients == single-process large
batch, bucketed/overlapped reducer, SyncBatchNorm == global-batch BN, metric reduction, driver."""

import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from jumbo_mae_tpu_amd.config import DecoderConfig, ViTConfig


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from jumbo_mae_tpu_amd.parallel import dist as pdist
    return pdist.init_distributed("cpu")


def _cfgs():
    vc = ViTConfig(layers=2, dim=32, heads=4, labels=0, image_size=32, patch_size=8, posemb="sincos2d",
                   layerscale=True)
    dc = DecoderConfig(dec_layers=2, dec_dim=16, dec_heads=2, image_size=32, patch_size=8)
    return vc, dc


def _dp_worker(rank, world, port, out, bucket_mb, defer=False, bf16=False):
    _init(rank, world, port)
    from jumbo_mae_tpu_amd.ops import prims
    prims._deferred["force"] = defer  # batched jumbo wgrad + chunked partial all-reduce (GPU path)
    partial = []
    from jumbo_mae_tpu_amd.models.mae import PretrainModel
    from jumbo_mae_tpu_amd.parallel.ddp import GradReducer
    from jumbo_mae_tpu_amd.train.meter import AverageMeter
    vc, dc = _cfgs()
    m = PretrainModel(vc, dc).to("cpu", seed=rank)  # different init per rank ...
    dist.broadcast(m.store.master, 0)               # ... made identical by the CC6 broadcast
    red = GradReducer(m.store, bucket_mb=bucket_mb, reduce_dtype=torch.bfloat16 if bf16 else torch.float32)
    m.store.partial_hooks.append(lambda h, lo, hi: partial.append((lo, hi)))
    g = torch.Generator().manual_seed(0)
    imgs = torch.randint(0, 256, (8, 3, 32, 32), dtype=torch.uint8, generator=g)
    noise = torch.rand(16, generator=g)
    mine = imgs[rank * 4:(rank + 1) * 4]
    m.store.zero_grad()
    red.begin_step()
    loss = m(mine, noise=noise)["loss"]
    loss.backward()
    launched_early = sum(red.launched)
    partial_launched = sum(1 for wk in red.works if wk[-1])  # partial slices issued before finish()
    stage = red.staging()
    stage_ptr = stage.data_ptr() if stage is not None else 0
    red.finish()
    meter = AverageMeter()
    meter.update(loss=loss.detach())
    summ = meter.summary()
    if rank == 0:
        same_stage = stage is None or red.staging().data_ptr() == stage_ptr  # no per-step allocation
        torch.save({"grad": m.store.grad.clone(), "launched_early": launched_early, "nb": len(red.buckets),
                    "partial": len(partial), "partial_launched": partial_launched, "same_stage": same_stage,
                    "loss": summ["loss"], "master": m.store.master.clone()}, out)
    dist.destroy_process_group()


@pytest.mark.parametrize("bucket_mb,defer,bf16", [(64.0, False, False), (0.01, False, False), (0.01, True, False),
                                                   (0.01, True, True)])
def test_dp_grads_equal_large_batch(bucket_mb, defer, bf16):
    from jumbo_mae_tpu_amd.models.mae import PretrainModel
    port = _free_port()
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "r.pt")
        mp.spawn(_dp_worker, args=(2, port, out, bucket_mb, defer, bf16), nprocs=2, join=True)
        res = torch.load(out, weights_only=True)
    vc, dc = _cfgs()
    ref = PretrainModel(vc, dc).to("cpu", seed=0)
    assert torch.equal(ref.store.master, res["master"])
    g = torch.Generator().manual_seed(0)
    imgs = torch.randint(0, 256, (8, 3, 32, 32), dtype=torch.uint8, generator=g)
    noise = torch.rand(16, generator=g)
    loss = ref(imgs, noise=noise)["loss"]
    loss.backward()
    if bf16:  # each rank's gradient rounded to bf16 before the average
        err = (res["grad"] - ref.store.grad).norm() / ref.store.grad.norm()
        assert err < 1e-2, err
        assert res["same_stage"]
    else:
        assert torch.allclose(res["grad"], ref.store.grad, atol=1e-6, rtol=1e-4)
    assert abs(res["loss"] - loss.item()) < 1e-5
    if bucket_mb < 1:
        assert res["nb"] > 3 and res["launched_early"] > 0  # buckets reduced while backward still ran
    if defer:  # jumbo w1 / w2 gradients reduced in row chunks as their batched GEMM writes them
        assert res["partial"] == 7  # w1: 4 chunks of 96 rows, w2: 3 chunks of 32
        # ... and launched as they are written -- before finish() -- with fp32 or bf16 reduction
        assert res["partial_launched"] == 7


def _bn_worker(rank, world, port, out):
    _init(rank, world, port)
    from jumbo_mae_tpu_amd.models.params import ParamStore, ones_, zeros_
    from jumbo_mae_tpu_amd.parallel.syncbn import sync_batch_norm
    s = ParamStore()
    hs = s.handle(s.add(("scale",), (6,), ones_))
    hb = s.handle(s.add(("bias",), (6,), zeros_))
    s.finalize("cpu")
    with torch.no_grad():
        s.master[:6] = torch.linspace(0.5, 2.0, 6)
    g = torch.Generator().manual_seed(1)
    x = torch.randn(8, 6, generator=g) * 3 + 1
    xm = x[rank * 4:(rank + 1) * 4].clone().requires_grad_()
    rm, rv = torch.zeros(6), torch.ones(6)
    y = sync_batch_norm(xm, hs, hb, rm, rv, training=True)
    w = torch.arange(48.0).view(8, 6)[rank * 4:(rank + 1) * 4] / 10
    (y * w).sum().backward()
    ys = [torch.zeros_like(y) for _ in range(2)]
    dist.all_gather(ys, y.detach())
    dxs = [torch.zeros_like(xm) for _ in range(2)]
    dist.all_gather(dxs, xm.grad)
    dist.all_reduce(s.grad)
    if rank == 0:
        torch.save({"y": torch.cat(ys), "dx": torch.cat(dxs), "gs": s.grad[:6].clone(), "gb": s.grad[6:12].clone(),
                    "rm": rm, "rv": rv}, out)
    dist.destroy_process_group()


def test_sync_batchnorm_equals_global_bn():
    port = _free_port()
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "bn.pt")
        mp.spawn(_bn_worker, args=(2, port, out), nprocs=2, join=True)
        r = torch.load(out, weights_only=True)
    g = torch.Generator().manual_seed(1)
    x = (torch.randn(8, 6, generator=g) * 3 + 1).requires_grad_()
    scale = torch.linspace(0.5, 2.0, 6).requires_grad_()
    bias = torch.zeros(6, requires_grad=True)
    mean = x.mean(0)
    var = (x * x).mean(0) - mean * mean
    y = (x - mean) / torch.sqrt(var + 1e-5) * scale + bias
    (y * (torch.arange(48.0).view(8, 6) / 10)).sum().backward()
    assert torch.allclose(r["y"], y, atol=1e-5)
    assert torch.allclose(r["dx"], x.grad, atol=1e-4)
    assert torch.allclose(r["gs"], scale.grad, atol=1e-4)
    assert torch.allclose(r["gb"], bias.grad, atol=1e-4)
    assert torch.allclose(r["rm"], 0.01 * mean.detach(), atol=1e-6)
    assert torch.allclose(r["rv"], 0.99 + 0.01 * var.detach(), atol=1e-5)


def _driver_worker(rank, world, port, outdir):
    _init(rank, world, port)
    from jumbo_mae_tpu_amd.train.cli import pretrain_parser
    from jumbo_mae_tpu_amd.train.pretrain import main
    args = pretrain_parser().parse_args([
        "--train-dataset-shards", "synthetic:64", "--valid-dataset-shards", "synthetic:12",
        "--train-batch-size", "8", "--valid-batch-size", "4", "--train-loader-workers", "0",
        "--valid-loader-workers", "0", "--auto-augment", "none", "--random-erasing", "0", "--augment-repeats", "1",
        "--layers", "1", "--dim", "32", "--heads", "2", "--labels", "0", "--image-size", "32", "--patch-size", "8",
        "--dec-layers", "1", "--dec-dim", "16", "--dec-heads", "2", "--training-steps", "4", "--warmup-steps", "1",
        "--log-interval", "2", "--eval-interval", "4", "--output-dir", outdir, "--name", "dd", "--grad-accum", "2",
        "--init-seed", "0", "--log-file-only"])
    res = main(args)
    if rank == 0:
        torch.save(res, os.path.join(outdir, "res.pt"))
    dist.destroy_process_group()


def test_pretrain_driver_two_ranks_grad_accum():
    port = _free_port()
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_driver_worker, args=(2, port, d), nprocs=2, join=True)
        res = torch.load(os.path.join(d, "res.pt"), weights_only=True)
        assert "val/loss" in res and res["val/loss"] > 0
        assert os.path.exists(os.path.join(d, "dd-last.msgpack"))
        assert os.path.exists(os.path.join(d, "dd-best.msgpack"))


def test_allreduce_bench_gloo(tmp_path):
    """tools/allreduce_bench.py (collective bandwidth sweep) runs on 2 gloo ranks and reports
    all-reduce / reduce-scatter / all-gather bus bandwidth plus the ViT-L exposure model."""
    import json
    import subprocess
    import sys

    out = tmp_path / "sweep.json"
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "tools", "allreduce_bench.py"), "--cpu", "--world", "2",
                        "--sizes-mb", "0.25,1", "--iters", "2", "--warmup", "1", "--port", str(_free_port()),
                        "--json", str(out)], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    res = json.loads(out.read_text())
    assert res["backend"] == "gloo" and len(res["collective_sweep"]) == 2
    for row in res["collective_sweep"]:
        assert row["world"] == 2
        assert row["allreduce_busbw_GBs"] > 0 and row["reduce_scatter_busbw_GBs"] > 0 and row["all_gather_busbw_GBs"] > 0
    assert res["model"]["vit_l_grad_allreduce_ms"] > res["model"]["vit_l_jumbo_tail_ms"] > 0
    assert res["model"]["recommended_bucket_mb"] in [row["size_mb"] for row in res["collective_sweep"]]


def _overlap_worker(rank, world, port, out, kind):
    _init(rank, world, port)
    from jumbo_mae_tpu_amd.models.mae import PretrainModel
    from jumbo_mae_tpu_amd.optim.flat import FlatOptimizer
    from jumbo_mae_tpu_amd.optim.schedule import warmup_cosine_decay_schedule
    from jumbo_mae_tpu_amd.parallel.ddp import GradReducer
    from jumbo_mae_tpu_amd.train.engine import Trainer
    vc, dc = _cfgs()
    g = torch.Generator().manual_seed(0)
    imgs = torch.randint(0, 256, (8, 3, 32, 32), dtype=torch.uint8, generator=g)
    res = {}
    for overlap in (False, True):
        torch.manual_seed(100 + rank)  # same masking noise in both runs
        m = PretrainModel(vc, dc).to("cpu", seed=0)
        dist.broadcast(m.store.master, 0)
        opt = FlatOptimizer(m.store, kind, warmup_cosine_decay_schedule(1e-6, 1e-2, 1, 10, 1e-5), b2=0.95,
                            weight_decay=0.05, num_layers=vc.layers)
        red = GradReducer(m.store, bucket_mb=0.01)
        tr = Trainer(m, opt, red, None)
        tr.overlap_optimizer = overlap
        calls = []
        real = opt.launch_range
        opt.launch_range = lambda lo, hi: (calls.append((lo, hi)), real(lo, hi))
        for step in range(3):
            tr.train_step([(imgs[rank * 4:(rank + 1) * 4],)])
        res[overlap] = (m.store.master.clone(), len(calls), len(red.optimizer_ranges()))
    if rank == 0:
        torch.save({"off": res[False][0], "on": res[True][0], "calls_on": res[True][1], "calls_off": res[False][1],
                    "nb": res[True][2]}, out)
    dist.destroy_process_group()


@pytest.mark.parametrize("kind", ["adamw", "sgd"])
def test_optimizer_overlaps_reduction_tail(kind):
    """Split optimizer step (each DP bucket updated as soon as its all-reduce is waited for, the
    rest at the end) == the monolithic step after the last reduction, bit for bit."""
    port = _free_port()
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "r.pt")
        mp.spawn(_overlap_worker, args=(2, port, out, kind), nprocs=2, join=True)
        res = torch.load(out, weights_only=True)
    assert res["calls_off"] == 0 and res["calls_on"] == 3 * res["nb"] and res["nb"] > 1
    assert torch.equal(res["on"], res["off"])
