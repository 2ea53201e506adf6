#!/usr/bin/env python3
"""Headline benchmark: Jumbo-MAE pretraining throughput (images/sec, whole job).

Metric/config from BASELINE.json: "pretrain images/sec (whole node) ViT-L/16 224 mask75% at
1/2/4/8 MI355X" -- ViT-L/16 Jumbo encoder (24 x 1024, 16 heads, 3 CLS tokens, shared jumbo
MLP), MAE decoder 8 x 512 (16 heads), mask ratio 0.75, AdamW(0.9, 0.95) + warmup-cosine with the
reference preset (config/pretrain/pretrain-vit-l16-224-in1k-800ep.sh), bf16 compute / fp32
master weights.  The reference preset's global batch of 4096 images per optimizer step is kept at
every N (strong scaling): 512 images per GPU on 8 GPUs, 1024 on 4, 2048 on 2, and on one GPU
2 x 2048 accumulated micro-batches -- the global batch fits in one MI355X's 288 GB (peak ~174 GB at
a 2048 micro-batch).  ``--batch-per-gpu B`` fixes the per-GPU batch instead (weak scaling).
Data: synthetic uint8 224x224 images resident on the GPU, random-init weights
(no datasets/checkpoints offline).  Every timed step is a full train step: forward, backward,
RCCL gradient all-reduce, optimizer update.

  python bench.py [--gpus N] [--steps K] [--warmup W]
  torchrun --nproc-per-node N bench.py --gpus N ...   (driver launches N>1 like this)

Secondary BASELINE.json configs (not the headline): ``--task finetune`` = ViT-B/16 end-to-end
finetune with the config/ft.sh recipe (AdamW + LLRD 0.75, Mixup 0.8 / CutMix 1.0, label
smoothing 0.1, droppath 0.1; global batch 1024 = 128 per GPU at 8 GPUs); ``--task linear`` =
ViT-L/16 linear probe with the LARS recipe (frozen encoder, SyncBatchNorm + Dense head; global
batch 16384 = 2048 per GPU at 8 GPUs).  Same synthetic-data / timing contract.
"""

from __future__ import annotations

import argparse
import json
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
    ap.add_argument("--global-batch", type=int, default=4096,
                    help="images per optimizer step over the whole job (reference preset: 4096)")
    ap.add_argument("--batch-per-gpu", type=int, default=0,
                    help="images per GPU per step; 0 (default) = global-batch / N (strong scaling); a value "
                         "fixes the per-GPU work at every N (weak scaling)")
    ap.add_argument("--max-micro-batch", type=int, default=2048,
                    help="largest micro-batch per GPU (HBM: ~174 GB at 2048 for ViT-L); a larger per-GPU batch "
                         "runs as gradient accumulation")
    ap.add_argument("--grad-accum", type=int, default=0, help="micro-steps per step (0: derived)")
    ap.add_argument("--grad-ckpt", action="store_true", help="activation checkpointing per layer (memory table)")
    ap.add_argument("--bucket-mb", type=float, default=64.0)
    ap.add_argument("--reduce-dtype", default="fp32", choices=["fp32", "bf16"],
                    help="gradient all-reduce dtype (fp32 master weights either way)")
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--shard-optimizer", action="store_true",
                    help="ZeRO-1: reduce-scatter + sharded optimizer + all-gather (default: all-reduce)")
    ap.add_argument("--zero1-gather", default="bf16", choices=["bf16", "fp32"],
                    help="ZeRO-1 weight all-gather dtype (bf16 shadow, or the fp32 master re-cast)")
    ap.add_argument("--profile-steps", type=int, default=0, help="extra steps under torch.profiler (debug)")
    ap.add_argument("--task", default="pretrain", choices=["pretrain", "finetune", "linear"])
    ap.add_argument("--dropout", type=float, default=0.0,
                    help="finetune: dropout rate of the attention / FF layers (config/ft.sh uses 0)")
    ap.add_argument("--cls-global-batch", type=int, default=0,
                    help="finetune / linear: images per step over the job; 0 = the reference preset "
                         "(config/ft.sh 1024, LARS linear probe 16384), split over N GPUs (strong scaling)")
    ap.add_argument("--hip-graph", action="store_true",
                    help="replay the captured train step from a HIP graph (single process; runtime/graph.py)")
    ap.add_argument("--cpu", action="store_true",
                    help="tests only: run the same flow on the CPU (gloo when distributed, fp32 PyTorch path)")
    ap.add_argument("--image-size", type=int, default=224, help=argparse.SUPPRESS)  # tests: smaller images
    args = ap.parse_args()
    if args.task != "pretrain":
        return bench_classifier(args)

    from jumbo_mae_tpu_amd.config import decoder_config, vit_config
    from jumbo_mae_tpu_amd.models.mae import PretrainModel
    from jumbo_mae_tpu_amd.optim.flat import FlatOptimizer
    from jumbo_mae_tpu_amd.optim.schedule import warmup_cosine_decay_schedule
    from jumbo_mae_tpu_amd.parallel import dist as pdist
    from jumbo_mae_tpu_amd.parallel.ddp import GradReducer
    from jumbo_mae_tpu_amd.train.engine import Trainer
    from jumbo_mae_tpu_amd.utils.flops import mfu, pretrain_fwd_flops_per_image
    from jumbo_mae_tpu_amd.utils.rng import RngStreams

    info = pdist.init_distributed("cpu" if args.cpu else None)
    dev = info.device
    world = info.world_size
    cdt = torch.float32 if args.cpu else torch.bfloat16
    if world != args.gpus and info.is_main:
        log(f"[bench] warning: --gpus {args.gpus} but WORLD_SIZE={world}; reporting WORLD_SIZE")
    # strong scaling by default: the reference's global batch 4096 at every N -- 2 x 2048 accumulated
    # micro-batches on 1 GPU (the global batch fitting in one MI355X's HBM), 2048 / 1024 / 512 per GPU
    # on 2 / 4 / 8 GPUs; --batch-per-gpu fixes the per-GPU batch instead (weak scaling)
    strong = args.batch_per_gpu == 0
    B = args.global_batch // world if strong else args.batch_per_gpu
    if strong and B * world != args.global_batch:
        raise SystemExit(f"global batch {args.global_batch} does not split over {world} ranks")
    if args.grad_accum <= 0:
        args.grad_accum = max(1, -(-B // args.max_micro_batch))
    if B % args.grad_accum:
        raise SystemExit(f"batch {B} per GPU does not split into {args.grad_accum} micro-batches")
    global_batch = B * world

    vc = vit_config(args.model, labels=0, posemb="sincos2d", image_mask_ratio=0.75, droppath=0.0, dropout=0.0,
                    image_size=args.image_size, grad_ckpt=args.grad_ckpt)
    dc = decoder_config(dec_droppath=0.0, image_size=args.image_size, grad_ckpt=args.grad_ckpt)
    model = PretrainModel(vc, dc).to(dev, cdt, seed=0)
    store = model.store
    pdist.broadcast_(store.master)  # CC6: identical init on every rank
    store.sync_shadow()
    # reference preset: lr 1.5e-4 * B/256, warmup 40 ep, 800 ep @ 4096 (pretrain-vit-l16-...-800ep.sh)
    steps_total = 1281167 * 800 // 4096
    sched = warmup_cosine_decay_schedule(1e-6, 1.5e-4 * 4096 / 256, 1281167 * 40 // 4096, steps_total, 1e-5)
    opt = FlatOptimizer(store, "adamw", sched, b1=0.9, b2=0.95, eps=1e-8, weight_decay=0.05,
                        num_layers=vc.layers)
    rdt = torch.bfloat16 if args.reduce_dtype == "bf16" else torch.float32
    reducer = (GradReducer(store, bucket_mb=args.bucket_mb, overlap=not args.no_overlap, reduce_dtype=rdt,
                           shard=args.shard_optimizer, gather_dtype=args.zero1_gather)
               if world > 1 or pdist.forced_group() else None)
    rngs = RngStreams({"noise": 0, "dropout": 0, "mixup": 0}, info.rank, dev)
    trainer = Trainer(model, opt, reducer, rngs, grad_accum=args.grad_accum)
    from jumbo_mae_tpu_amd.runtime.graph import StepRunner
    runner = StepRunner(trainer, hip_graph=args.hip_graph and world == 1)

    gen = torch.Generator(device=dev).manual_seed(1234 + info.rank)
    mb = B // args.grad_accum
    S = args.image_size
    pool = [torch.randint(0, 256, (mb, 3, S, S), dtype=torch.uint8, device=dev, generator=gen) for _ in range(2)]

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
        return runner(micro)

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()

    t0 = time.time()
    for i in range(args.warmup):
        m = step()
        if info.is_main:
            sync()
            log(f"[bench] warmup {i + 1}/{args.warmup} loss={m['loss'].item():.4f} lr={m['learning_rate']:.3e} "
                f"t={time.time() - t0:.1f}s")
    pdist.barrier()
    sync()
    t_start = time.perf_counter()
    for i in range(args.steps):
        m = step()
        if info.is_main and (i + 1) % max(1, args.steps // 4) == 0:
            log(f"[bench] step {i + 1}/{args.steps} t={time.perf_counter() - t_start:.2f}s")
    pdist.barrier()
    sync()
    elapsed = time.perf_counter() - t_start
    elapsed = pdist.all_reduce_max_scalar(elapsed, dev)
    final_loss = float(m["loss"].item())
    comm_ms = trainer.comm_ms()
    # multi-GPU self-calibration, outside the timed region: one traced step (when each bucket's
    # gradient became final, on the GPU clock) and one timed collective per distinct bucket size
    # of the real plan -- the inputs of tools/dp_exposure_model.py (--sweep reads this JSON line)
    calib = trace_and_calibrate(reducer, step, dev) if (reducer is not None and world > 1) else None
    if reducer is not None and reducer.shard:
        opt.gather_state()  # ZeRO-1: the sharded fp32 master (and moments) made whole for the checksum
    # data-parallel replicas must hold identical weights after the timed steps (outside the timed
    # region): spread of a weight checksum over the ranks, 0.0 when in sync
    spread = pdist.all_reduce_max_scalar(float(store.master.double().abs().sum()), dev) - \
        -pdist.all_reduce_max_scalar(-float(store.master.double().abs().sum()), dev) if world > 1 else 0.0
    weight_checksum = float(store.master.double().abs().sum())

    if args.profile_steps > 0 and info.is_main:
        from torch.profiler import ProfilerActivity, profile
        stacks = ""
        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=bool(stacks)) as prof:
            for _ in range(args.profile_steps):
                step()
            sync()
        log(prof.key_averages().table(sort_by="cuda_time_total", row_limit=150))
        if stacks:
            for ev in prof.key_averages(group_by_stack_n=6):
                if ev.key in stacks.split(","):
                    log(f"{ev.key} x{ev.count} {ev.device_time_total:.0f}us <- " + " | ".join(ev.stack[:6]))

    ms = elapsed / args.steps * 1000.0
    value = global_batch * args.steps / elapsed
    peak_gb = round(torch.cuda.max_memory_allocated(dev) / 2**30, 2) if dev.type == "cuda" else None
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
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "mfu_bf16_dense": round(mfu(value, pretrain_fwd_flops_per_image(vc, dc), world), 4),
            # GPU time of the last step behind the DP reduction wait (exposed comm + overlapped
            # bucket updates); null on one GPU
            "exposed_comm_ms_last_step": None if comm_ms is None else round(comm_ms, 3),
            # peak HBM held by PyTorch's allocator on this rank (torch.cuda.max_memory_allocated)
            "peak_hbm_gb": peak_gb,
            "replica_weight_checksum_spread": spread, "weight_checksum": weight_checksum,
            "reducer": reducer.stats() if reducer is not None else None,
            **(calib or {}),
            "dtype": "fp32" if args.cpu else "bf16",
            "data": f"synthetic uint8 {S}x{S} images on {'CPU' if args.cpu else 'GPU'}, random-init weights",
            "config": {
                "model": f"{args.model} jumbo-MAE (3 CLS, shared jumbo MLP) + decoder 8x512x16h",
                "global_batch": global_batch,
                "seq_len": vc.num_cls_tokens + vc.keep_len,
                "decoder_seq_len": vc.num_cls_tokens + vc.seq_patches,
                "parallelism": f"dp{world}",
                "per_gpu_batch": B,
                "grad_accum": args.grad_accum,
                "micro_batch": mb,
                "grad_ckpt": args.grad_ckpt,
                "hip_graph": bool(runner.graphed is not None),
                "optimizer": "adamw(0.9,0.95) wd0.05 warmup-cosine",
                "final_loss": round(final_loss, 5),
            },
        }
        print(json.dumps(out), flush=True)
    pdist.cleanup()


def trace_and_calibrate(reducer, step, dev) -> dict:
    """One extra (untimed) step with the reducer's readiness trace on -> per-collective ready times
    relative to the step start; then ``parallel.collbench.calibrate`` on the same process group."""
    import time as _t

    from jumbo_mae_tpu_amd.parallel.collbench import calibrate
    cuda = dev.type == "cuda"
    reducer.trace_events = []
    if cuda:
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
    h0 = _t.perf_counter()
    step()
    if cuda:
        e1.record()
        torch.cuda.synchronize()
    esz = 2 if reducer.reduce_dtype == torch.bfloat16 else 4
    spans = []
    for b, lo, hi, partial, ev in reducer.trace_events:
        t = e0.elapsed_time(ev) if cuda else (ev - h0) * 1e3
        spans.append({"bucket": b, "bytes": (hi - lo) * esz, "ready_ms": round(t, 3), "partial": bool(partial)})
    reducer.trace_events = None
    step_ms = e0.elapsed_time(e1) if cuda else (_t.perf_counter() - h0) * 1e3
    return {"dp_traced_step_ms": round(step_ms, 3), "dp_ready_spans": spans,
            "collective_sweep": calibrate(reducer, dev)}


def bench_classifier(args):
    """Finetune (ViT-B/16, config/ft.sh) or linear probe (ViT-L/16, LARS preset) step throughput."""
    from jumbo_mae_tpu_amd.parallel import dist as pdist
    from jumbo_mae_tpu_amd.train import common as C
    from jumbo_mae_tpu_amd.train.cli import finetune_parser
    from jumbo_mae_tpu_amd.train.engine import Trainer
    from jumbo_mae_tpu_amd.train.finetune import build_model
    from jumbo_mae_tpu_amd.utils.flops import finetune_fwd_flops_per_image, mfu
    from jumbo_mae_tpu_amd.utils.rng import RngStreams

    info = pdist.init_distributed()
    dev = info.device
    world = info.world_size
    N = 1281167
    strong = not args.batch_per_gpu
    gb_ref = args.cls_global_batch or (1024 if args.task == "finetune" else 16384)
    if strong and gb_ref % world:
        raise SystemExit(f"global batch {gb_ref} is not divisible by {world} GPUs")
    B = args.batch_per_gpu or gb_ref // world
    gb = B * world
    accum = -(-B // max(1, args.max_micro_batch))
    while B % accum:
        accum += 1
    micro = B // accum
    if args.task == "finetune":
        flags = ["--mode", "finetune", "--layers", "12", "--dim", "768", "--heads", "12", "--labels", "1000",
                 "--posemb", "sincos2d", "--droppath", "0.1", "--dropout", str(args.dropout),
                 "--mixup", "0.8", "--cutmix", "1.0",
                 "--label-smoothing", "0.1", "--optimizer", "adamw", "--learning-rate", "3e-3",
                 "--weight-decay", "0.05", "--lr-decay", "0.75", "--warmup-steps", str(N * 10 // 1024),
                 "--training-steps", str(N * 110 // 1024)]
        model_name = "vit_base_patch16 jumbo (3 CLS) finetune"
        recipe = "adamw llrd0.75 mixup0.8 cutmix1.0 ls0.1 dp0.1" + (f" dropout{args.dropout}" if args.dropout else "")
    else:
        flags = ["--mode", "linear", "--layers", "24", "--dim", "1024", "--heads", "16", "--labels", "1000",
                 "--posemb", "sincos2d", "--droppath", "0.0", "--mixup", "0.0", "--cutmix", "0.0",
                 "--label-smoothing", "0.0", "--optimizer", "lars", "--learning-rate", "0.1",
                 "--weight-decay", "0.0", "--warmup-steps", str(N * 10 // 16384),
                 "--training-steps", str(N * 90 // 16384)]
        model_name, recipe = "vit_large_patch16 jumbo (3 CLS) linear probe", "lars syncbn-head"
    # fixed seeds (the CLI defaults them to random.randint, as the reference does): reproducible runs
    for k in ("init", "mixup", "dropout", "shuffle", "noise"):
        flags += [f"--{k}-seed", "0"]
    fargs = finetune_parser().parse_args(flags + ["--train-batch-size", str(gb), "--bucket-mb", str(args.bucket_mb),
                                                "--reduce-dtype", args.reduce_dtype]
                                         + (["--shard-optimizer", "--zero1-gather", args.zero1_gather]
                                            if args.shard_optimizer else []))
    model = build_model(fargs, dev, torch.bfloat16, info.rank)
    pdist.broadcast_(model.store.master)
    model.store.sync_shadow()
    peak = fargs.learning_rate * gb / 256 if fargs.optimizer == "lars" else fargs.learning_rate
    import contextlib
    with contextlib.redirect_stdout(sys.stderr):  # stdout carries only the JSON result line
        opt = C.make_optimizer(fargs, model.store, peak, 1e-6)
    reducer = C.make_reducer(fargs, model.store)
    rngs = RngStreams({"mixup": 1, "dropout": 1, "noise": 1}, info.rank, dev)
    trainer = Trainer(model, opt, reducer, rngs)
    from jumbo_mae_tpu_amd.runtime.graph import StepRunner
    runner = StepRunner(trainer, hip_graph=args.hip_graph and world == 1)
    gen = torch.Generator(device=dev).manual_seed(1234 + info.rank)
    pool = [(torch.randint(0, 256, (micro, 3, 224, 224), dtype=torch.uint8, device=dev, generator=gen),
             torch.randint(0, 1000, (micro,), device=dev, generator=gen)) for _ in range(2)]
    if info.is_main:
        log(f"[bench] task={args.task} params={model.store.num_params()/1e6:.1f}M "
            f"trainable={model.store.num_params(True)/1e6:.2f}M world={world} batch/gpu={B} = {accum} x {micro}")
    it = 0

    def step():
        nonlocal it
        m = runner([pool[(it + j) % 2] for j in range(accum)])
        it += 1
        return m

    for i in range(args.warmup):
        m = step()
        if info.is_main:
            torch.cuda.synchronize()
            log(f"[bench] warmup {i + 1}/{args.warmup} loss={m['loss'].item():.4f}")
    pdist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        m = step()
    pdist.barrier()
    torch.cuda.synchronize()
    elapsed = pdist.all_reduce_max_scalar(time.perf_counter() - t0, dev)
    value = gb * args.steps / elapsed
    fwd = finetune_fwd_flops_per_image(model.cfg)
    util = mfu(value, fwd, world) if args.task == "finetune" else mfu(value, fwd, world) / 3.0
    if info.is_main:
        print(json.dumps({
            "metric": f"{args.task} images/sec (whole node) " + ("ViT-B/16" if args.task == "finetune" else "ViT-L/16")
            + " 224",
            "value": round(value, 2), "unit": "images/sec", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1000.0, 3),
            "higher_is_better": True, "scaling": "strong" if strong else "weak", "vs_baseline": None,
            "mfu_bf16_dense": round(util, 4), "dtype": "bf16",
            "reducer": reducer.stats() if reducer is not None else None,
            "peak_hbm_gb": round(torch.cuda.max_memory_allocated(dev) / 2**30, 2),
            "data": "synthetic uint8 224x224 images + random labels on GPU, random-init weights",
            "config": {"model": model_name, "global_batch": gb, "seq_len": model.cfg.num_cls_tokens
                       + model.cfg.seq_patches, "parallelism": f"dp{world}", "per_gpu_batch": B,
                       "micro_batch": micro, "grad_accum": accum,
                       "hip_graph": bool(runner.graphed is not None),
                       "recipe": recipe, "final_loss": round(float(m["loss"].item()), 5)},
        }), flush=True)
    pdist.cleanup()


if __name__ == "__main__":
    main()
