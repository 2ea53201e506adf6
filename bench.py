#!/usr/bin/env python3
"""Headline benchmark: Jumbo-MAE pretraining throughput (images/sec, whole job).

Metric/config from BASELINE.json: "pretrain images/sec (whole node) ViT-L/16 224 mask75% at
1/2/4/8 MI355X" -- ViT-L/16 Jumbo encoder (24 x 1024, 16 heads, 3 CLS tokens, shared jumbo
MLP), MAE decoder 8 x 512 (16 heads), mask ratio 0.75, AdamW(0.9, 0.95) + warmup-cosine with the
reference preset (config/pretrain/pretrain-vit-l16-224-in1k-800ep.sh), bf16 compute / fp32
master weights.  Global batch 4096 on 8 GPUs = 512 images per GPU; weak scaling keeps 512 per
GPU at every N.  Data: synthetic uint8 224x224 images resident on the GPU, random-init weights
(no datasets/checkpoints offline).  Every timed step is a full train step: forward, backward,
RCCL gradient all-reduce, optimizer update.

  python bench.py [--gpus N] [--steps K] [--warmup W]
  torchrun --nproc-per-node N bench.py --gpus N ...   (driver launches N>1 like this)
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--model", default="vit_large_patch16", choices=["vit_large_patch16", "vit_base_patch16",
                                                                      "vit_small_patch16", "vit_tiny_patch16"])
    ap.add_argument("--batch-per-gpu", type=int, default=512)
    ap.add_argument("--grad-accum", type=int, default=1)
    ap.add_argument("--bucket-mb", type=float, default=64.0)
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--profile-steps", type=int, default=0, help="extra steps under torch.profiler (debug)")
    args = ap.parse_args()

    from jumbo_mae_tpu_amd.config import decoder_config, vit_config
    from jumbo_mae_tpu_amd.models.mae import PretrainModel
    from jumbo_mae_tpu_amd.optim.flat import FlatOptimizer
    from jumbo_mae_tpu_amd.optim.schedule import warmup_cosine_decay_schedule
    from jumbo_mae_tpu_amd.parallel import dist as pdist
    from jumbo_mae_tpu_amd.parallel.ddp import GradReducer
    from jumbo_mae_tpu_amd.train.engine import Trainer
    from jumbo_mae_tpu_amd.utils.flops import mfu, pretrain_fwd_flops_per_image
    from jumbo_mae_tpu_amd.utils.rng import RngStreams

    info = pdist.init_distributed()
    dev = info.device
    world = info.world_size
    if world != args.gpus and info.is_main:
        log(f"[bench] warning: --gpus {args.gpus} but WORLD_SIZE={world}; reporting WORLD_SIZE")
    B = args.batch_per_gpu
    global_batch = B * world

    vc = vit_config(args.model, labels=0, posemb="sincos2d", image_mask_ratio=0.75, droppath=0.0, dropout=0.0)
    dc = decoder_config(dec_droppath=0.0)
    model = PretrainModel(vc, dc).to(dev, torch.bfloat16, seed=0)
    store = model.store
    pdist.broadcast_(store.master)  # CC6: identical init on every rank
    store.sync_shadow()
    # reference preset: lr 1.5e-4 * B/256, warmup 40 ep, 800 ep @ 4096 (pretrain-vit-l16-...-800ep.sh)
    steps_total = 1281167 * 800 // 4096
    sched = warmup_cosine_decay_schedule(1e-6, 1.5e-4 * 4096 / 256, 1281167 * 40 // 4096, steps_total, 1e-5)
    opt = FlatOptimizer(store, "adamw", sched, b1=0.9, b2=0.95, eps=1e-8, weight_decay=0.05,
                        num_layers=vc.layers)
    reducer = GradReducer(store, bucket_mb=args.bucket_mb, overlap=not args.no_overlap) if world > 1 else None
    rngs = RngStreams({"noise": 0, "dropout": 0, "mixup": 0}, info.rank, dev)
    trainer = Trainer(model, opt, reducer, rngs, grad_accum=args.grad_accum)

    gen = torch.Generator(device=dev).manual_seed(1234 + info.rank)
    mb = B // args.grad_accum
    pool = [torch.randint(0, 256, (mb, 3, 224, 224), dtype=torch.uint8, device=dev, generator=gen)
            for _ in range(2)]

    if info.is_main:
        log(f"[bench] {args.model} jumbo-MAE params={store.num_params()/1e6:.1f}M world={world} "
            f"batch/gpu={B} accum={args.grad_accum} device={torch.cuda.get_device_name(dev) if dev.type == 'cuda' else 'cpu'}")
        if reducer is not None:
            log(f"[bench] reducer {reducer.stats()}")

    it = 0

    def step():
        nonlocal it
        micro = [(pool[(it + j) % 2],) for j in range(args.grad_accum)]
        it += 1
        return trainer.train_step(micro)

    t0 = time.time()
    for i in range(args.warmup):
        m = step()
        if info.is_main:
            torch.cuda.synchronize()
            log(f"[bench] warmup {i + 1}/{args.warmup} loss={m['loss'].item():.4f} lr={m['learning_rate']:.3e} "
                f"t={time.time() - t0:.1f}s")
    pdist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for i in range(args.steps):
        m = step()
        if info.is_main and (i + 1) % max(1, args.steps // 4) == 0:
            log(f"[bench] step {i + 1}/{args.steps} t={time.perf_counter() - t_start:.2f}s")
    pdist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    elapsed = pdist.all_reduce_max_scalar(elapsed, dev)
    final_loss = float(m["loss"].item())

    if args.profile_steps > 0 and info.is_main:
        from torch.profiler import ProfilerActivity, profile
        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
            for _ in range(args.profile_steps):
                step()
            torch.cuda.synchronize()
        log(prof.key_averages().table(sort_by="cuda_time_total", row_limit=40))

    ms = elapsed / args.steps * 1000.0
    value = global_batch * args.steps / elapsed
    if info.is_main:
        out = {
            "metric": "pretrain images/sec (whole node) ViT-L/16 224 mask75% at 1/2/4/8 MI355X"
            if args.model == "vit_large_patch16" else f"pretrain images/sec {args.model} 224 mask75%",
            "value": round(value, 2),
            "unit": "images/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "mfu_bf16_dense": round(mfu(value, pretrain_fwd_flops_per_image(vc, dc), world), 4),
            "dtype": "bf16",
            "data": "synthetic uint8 224x224 images on GPU, random-init weights",
            "config": {
                "model": f"{args.model} jumbo-MAE (3 CLS, shared jumbo MLP) + decoder 8x512x16h",
                "global_batch": global_batch,
                "seq_len": vc.num_cls_tokens + vc.keep_len,
                "decoder_seq_len": vc.num_cls_tokens + vc.seq_patches,
                "parallelism": f"dp{world}",
                "per_gpu_batch": B,
                "grad_accum": args.grad_accum,
                "optimizer": "adamw(0.9,0.95) wd0.05 warmup-cosine",
                "final_loss": round(final_loss, 5),
            },
        }
        print(json.dumps(out), flush=True)
    pdist.cleanup()


if __name__ == "__main__":
    main()
