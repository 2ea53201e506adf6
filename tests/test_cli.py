"""CLI parity: every reference preset command line and every one of our presets parses with our
argparse, with identical flag names/spellings."""

import glob
import os
import re
import subprocess

import pytest

from jumbo_mae_tpu_amd.train.cli import finetune_parser, pretrain_parser

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference/config"


def _reference_argv(path):
    text = open(path).read()
    m = re.search(r"python3 src/(main_\w+)\.py(.*?)(?:\n\s*done|\Z)", text, re.S)
    entry, body = m.group(1), m.group(2)
    body = body.replace("\\\n", " ")
    body = re.sub(r"\$\(\((.*?)\)\)", lambda mm: str(eval(mm.group(1).replace("/", "//"))), body)
    body = re.sub(r"\$\([^)]*\)", "x", body)
    body = body.replace("${lr}", "1e-3").replace("${wd}", "0.05")
    body = re.sub(r"\$\{?\w+\}?", "x", body)
    import shlex
    return entry, shlex.split(body)


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference presets not mounted")
@pytest.mark.parametrize("path", sorted(glob.glob(f"{REF}/**/*.sh", recursive=True)))
def test_reference_presets_parse(path):
    entry, argv = _reference_argv(path)
    parser = pretrain_parser() if entry == "main_pretrain" else finetune_parser()
    args = parser.parse_args(argv)
    assert args.train_batch_size > 0
    if entry == "main_pretrain":
        assert args.image_mask_ratio == 0.75 and args.dec_layers == 8


@pytest.mark.parametrize("path", sorted(glob.glob(f"{ROOT}/config/**/*.sh", recursive=True)))
def test_our_presets_dryrun(path):
    if os.path.basename(path).startswith("_"):
        return
    env = dict(os.environ, JMAE_DRYRUN="1", NGPU="8", PRETRAINED="/tmp/x.msgpack")
    out = subprocess.run(["bash", path], capture_output=True, text=True, env=env, timeout=120)
    assert out.returncode == 0, out.stderr
    lines = out.stdout.strip().split("\n")
    runs = [i for i, l in enumerate(lines) if l.endswith(".py")]
    assert runs, out.stdout
    for k, i in enumerate(runs):
        end = runs[k + 1] if k + 1 < len(runs) else len(lines)
        argv = [a for a in lines[i + 1:end] if not a.startswith("Running with")]
        parser = pretrain_parser() if lines[i] == "main_pretrain.py" else finetune_parser()
        args = parser.parse_args(argv)
        assert args.warmup_steps >= 0 and args.training_steps > 0


def test_defaults_match_reference():
    a = pretrain_parser().parse_args([])
    assert (a.train_batch_size, a.valid_batch_size, a.dec_layers, a.dec_heads, a.droppath) == (4096, 512, 6, 8, 0.1)
    assert (a.posemb, a.auto_augment, a.augment_repeats, a.learning_rate) == ("sincos2d", "rand-m9-mstd0.5-inc1", 3, 1e-3)
    f = finetune_parser().parse_args([])
    assert (f.train_batch_size, f.valid_batch_size, f.posemb, f.criterion, f.label_smoothing) == \
        (2048, 256, "learnable", "ce", 0.1)


def test_device_augment_auto_needs_the_extension(monkeypatch):
    """--device-augment auto falls back to the PIL path when the HIP extension is not built (a
    JMAE_ALLOW_TORCH_FALLBACK run); 'on' fails early with a clear message instead of inside the
    prefetcher."""
    from types import SimpleNamespace

    import torch

    from jumbo_mae_tpu_amd.ops import _ext
    from jumbo_mae_tpu_amd.train import common as C

    args = SimpleNamespace(device_augment="auto", train_dataset_shards="x-{0..1}.tar", random_crop="rrc",
                           auto_augment="none", color_jitter=0.0, random_erasing=0.0)
    cuda = torch.device("cuda")
    monkeypatch.setattr(_ext, "available", lambda: False)
    assert C.use_device_augment(args, cuda) is False
    args.device_augment = "on"
    with pytest.raises(SystemExit, match="extension"):
        C.use_device_augment(args, cuda)
    monkeypatch.setattr(_ext, "available", lambda: True)
    assert C.use_device_augment(args, cuda) is True
    args.device_augment = "auto"
    assert C.use_device_augment(args, torch.device("cpu")) is False
