"""Command-line flags, identical in name, spelling and default to the reference drivers.

Reference: /root/reference/src/main_pretrain.py:97-167 and main_finetune.py:97-160 (note the
underscore spelling of ``--image_mask_ratio`` and the seeds defaulting to ``random.randint`` at
parse time).  Additions (all optional, defaults keep reference behaviour): ``--resume``,
``--save-interval``, ``--mask-mode``, ``--compute-dtype``, ``--bucket-mb``, ``--device``.
Flags the reference accepts but ignores (``--pooling``, ``--dec-posemb``, ``--label-mapping``,
``--ipaddr``, ``--hostname``; quirk Q10) are accepted and recorded.
"""

from __future__ import annotations

import argparse
import random


def _common(p: argparse.ArgumentParser, mode: str, batch: int, vbatch: int, posemb: str):
    p.add_argument("--mode", default=mode)
    p.add_argument("--train-dataset-shards")
    p.add_argument("--valid-dataset-shards")
    p.add_argument("--train-batch-size", type=int, default=batch)
    p.add_argument("--valid-batch-size", type=int, default=vbatch)
    p.add_argument("--train-loader-workers", type=int, default=40)
    p.add_argument("--valid-loader-workers", type=int, default=5)

    p.add_argument("--random-crop", default="rrc")
    p.add_argument("--color-jitter", type=float, default=0.0)
    p.add_argument("--auto-augment", default="rand-m9-mstd0.5-inc1")
    p.add_argument("--random-erasing", type=float, default=0.25)
    p.add_argument("--augment-repeats", type=int, default=3)
    p.add_argument("--test-crop-ratio", type=float, default=0.875)

    p.add_argument("--mixup", type=float, default=0.8)
    p.add_argument("--cutmix", type=float, default=1.0)
    return p


def _model(p: argparse.ArgumentParser, posemb: str):
    p.add_argument("--layers", type=int, default=12)
    p.add_argument("--dim", type=int, default=768)
    p.add_argument("--heads", type=int, default=12)
    p.add_argument("--labels", type=int, default=-1)
    p.add_argument("--layerscale", action="store_true", default=False)
    p.add_argument("--patch-size", type=int, default=16)
    p.add_argument("--image-size", type=int, default=224)
    p.add_argument("--posemb", default=posemb)
    p.add_argument("--pooling", default="cls")
    p.add_argument("--dropout", type=float, default=0.0)
    p.add_argument("--droppath", type=float, default=0.1)
    p.add_argument("--grad-ckpt", action="store_true", default=False)


def _optim(p: argparse.ArgumentParser):
    p.add_argument("--optimizer", default="adamw")
    p.add_argument("--learning-rate", type=float, default=1e-3)
    p.add_argument("--weight-decay", type=float, default=0.05)
    p.add_argument("--adam-b1", type=float, default=0.9)
    p.add_argument("--adam-b2", type=float, default=0.999)
    p.add_argument("--adam-eps", type=float, default=1e-8)
    p.add_argument("--lr-decay", type=float, default=1.0)
    p.add_argument("--clip-grad", type=float, default=0.0)
    p.add_argument("--grad-accum", type=int, default=1)

    p.add_argument("--warmup-steps", type=int, default=10000)
    p.add_argument("--training-steps", type=int, default=200000)
    p.add_argument("--log-interval", type=int, default=50)
    p.add_argument("--eval-interval", type=int, default=0)

    p.add_argument("--project")
    p.add_argument("--name")
    p.add_argument("--ipaddr")
    p.add_argument("--hostname")
    p.add_argument("--output-dir", default=".", type=_output_dir)


def _output_dir(v: str) -> str:
    """Checkpoint names are joined onto the output dir, which a ``pipe:`` command cannot take (its
    read command would run with the checkpoint bytes on stdin and write nothing)."""
    if v.startswith("pipe:"):
        raise argparse.ArgumentTypeError("--output-dir cannot be a pipe: command; use a path or gs:// / s3:// URL")
    return v


def _extensions(p: argparse.ArgumentParser):
    g = p.add_argument_group("MI355X framework extensions")
    g.add_argument("--resume", default=None,
                   help="'auto' or a path prefix {output_dir}/{name}-last: resume params + optimizer + step")
    g.add_argument("--save-interval", type=int, default=0, help="also save 'last' every N steps (0: at eval)")
    g.add_argument("--compute-dtype", default="auto", choices=["auto", "bf16", "fp32"])
    g.add_argument("--bucket-mb", type=float, default=64.0,
                   help="data-parallel all-reduce bucket size (tools/allreduce_bench.py recommends one)")
    g.add_argument("--reduce-dtype", default="fp32", choices=["fp32", "bf16"],
                   help="gradient all-reduce dtype (bf16 halves the bytes on xGMI; master weights, "
                        "optimizer state and the local gradient stay fp32)")
    g.add_argument("--shard-optimizer", action="store_true",
                   help="ZeRO-1: reduce-scatter the gradient buckets, update 1/N of the parameters per rank, "
                        "all-gather the updated weights (parallel/ddp.py)")
    g.add_argument("--zero1-gather", default="bf16", choices=["bf16", "fp32"],
                   help="ZeRO-1 weight all-gather: the bf16 compute shadow (fp32 master stays sharded until a "
                        "checkpoint) or the fp32 master (re-cast after the gather)")
    g.add_argument("--stop-after-steps", type=int, default=0,
                   help="end this invocation after N steps, writing 'last' (time-sliced / preemptible "
                        "jobs: continue with --resume auto); 0 = run to --training-steps")
    g.add_argument("--device", default=None, help="cuda|cpu (default: cuda if available)")
    g.add_argument("--device-augment", default="auto", choices=["auto", "on", "off"],
                   help="RandomResizedCrop + flip of the train batches on the GPU, bit-exact to PIL (auto: on a GPU "
                        "when the train transform is exactly that -- the pretraining presets)")
    g.add_argument("--log-file-only", action="store_true", help="never use wandb even if installed")
    g.add_argument("--trace-ranges", action="store_true", help="roctx ranges per step phase (rocprofv3 --marker-trace)")
    g.add_argument("--hip-graph", action="store_true",
                   help="capture the whole train step once in a HIP graph and replay it (single process)")
    g.add_argument("--skip-nonfinite", action="store_true",
                   help="skip the update of a step whose loss is non-finite (one host sync per step); "
                        "default: abort at the next log step")


def pretrain_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser("main_pretrain")
    _common(p, "pretrain", 4096, 512, "sincos2d")
    # reference places --image_mask_ratio right after --mode (main_pretrain.py:100)
    p.add_argument("--image_mask_ratio", type=float, default=0.75)
    _model(p, "sincos2d")
    p.add_argument("--dec-layers", type=int, default=6)
    p.add_argument("--dec-dim", type=int, default=512)
    p.add_argument("--dec-heads", type=int, default=8)
    p.add_argument("--dec-layerscale", action="store_true", default=False)
    p.add_argument("--dec-posemb", default="sincos2d")
    p.add_argument("--dec-dropout", type=float, default=0.0)
    p.add_argument("--dec-droppath", type=float, default=0.1)
    p.add_argument("--norm-pix-loss", action="store_true", default=False)
    for s in ("init", "mixup", "dropout", "noise", "shuffle"):
        p.add_argument(f"--{s}-seed", type=int, default=random.randint(0, 1000000))
    _optim(p)
    _extensions(p)
    p.add_argument("--mask-mode", default="shared", choices=["shared", "per-sample"],
                   help="shared: one permutation per rank per step (reference, Q1)")
    return p


def finetune_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser("main_finetune")
    p.add_argument("--pretrained-ckpt", default=None)
    _common(p, "finetune", 2048, 256, "learnable")
    p.add_argument("--criterion", default="ce")
    p.add_argument("--label-smoothing", type=float, default=0.1)
    _model(p, "learnable")
    for s in ("init", "mixup", "dropout", "shuffle", "noise"):
        p.add_argument(f"--{s}-seed", type=int, default=random.randint(0, 1000000))
    p.add_argument("--label-mapping")
    _optim(p)
    _extensions(p)
    return p
