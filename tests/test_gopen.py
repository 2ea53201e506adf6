"""Remote URLs (gs://, s3://, http(s)://, pipe:) for shards, checkpoints and pretrained params,
through stub ``gsutil`` / ``curl`` executables on PATH that serve a local directory.

Reference: every preset reads and writes ``$GCS_DATASET_DIR/...`` = ``gs://...`` through
webdataset's gopen (/root/reference/src/utils.py:55-63,151; src/dataset.py:107-116;
config/ft.sh:3-6)."""

import os
import stat
import subprocess

import numpy as np
import pytest

from jumbo_mae_tpu_amd.ckpt.checkpoint import (ckpt_path, load_params, load_pretrained_params, save_params,
                                               write_bytes, writer)
from jumbo_mae_tpu_amd.config import ViTConfig
from jumbo_mae_tpu_amd.data import shards as S
from jumbo_mae_tpu_amd.data.loader import ShardDataset
from jumbo_mae_tpu_amd.data.transforms import create_transforms
from jumbo_mae_tpu_amd.models.classifier import FinetuneModel
from jumbo_mae_tpu_amd.utils import gopen

from test_ckpt import _pre
from test_data import _make_tar

GSUTIL = """#!/bin/bash
# gsutil stub: cat gs://b/p | cp - gs://b/p | -q stat gs://b/p, served from $STUB_ROOT/gs/b/p
root="$STUB_ROOT/gs"
case "$1" in
  cat) exec cat "$root/${2#gs://}" ;;
  cp) [ "$2" = "-" ] || exit 2; f="$root/${3#gs://}"; mkdir -p "$(dirname "$f")"; exec cat > "$f" ;;
  -q) [ "$2" = stat ] && test -f "$root/${3#gs://}" ;;
  *) exit 2 ;;
esac
"""

CURL = """#!/bin/bash
# curl stub: curl -fsSL <url> | curl -fsIL -o /dev/null <url>, served from $STUB_ROOT/http/<host/path>
url="${@: -1}"; f="$STUB_ROOT/http/${url#*://}"
[ -f "$f" ] || exit 22
if [ "$1" = "-fsSL" ]; then exec cat "$f"; fi
exit 0
"""


@pytest.fixture
def stub(tmp_path, monkeypatch):
    bindir = tmp_path / "bin"
    bindir.mkdir()
    for name, body in (("gsutil", GSUTIL), ("curl", CURL)):
        p = bindir / name
        p.write_text(body)
        p.chmod(p.stat().st_mode | stat.S_IEXEC)
    root = tmp_path / "remote"
    (root / "gs").mkdir(parents=True)
    (root / "http").mkdir(parents=True)
    monkeypatch.setenv("PATH", f"{bindir}:{os.environ['PATH']}")
    monkeypatch.setenv("STUB_ROOT", str(root))
    work = tmp_path / "work"
    work.mkdir()
    monkeypatch.chdir(work)  # a local "gs:" directory created by mistake would land here
    return root


def test_scheme_and_join():
    assert gopen.scheme("/a/b") == "" and gopen.scheme("file:///a") == ""
    assert gopen.scheme("pipe:cat x") == "pipe" and gopen.scheme("gs://b/x") == "gs"
    assert gopen.join("gs://b/CKPT", "x.msgpack") == "gs://b/CKPT/x.msgpack"
    assert gopen.join("gs://b/CKPT/", "x") == "gs://b/CKPT/x"
    assert ckpt_path("gs://b/CKPT", "run", "last") == "gs://b/CKPT/run-last.msgpack"
    assert gopen.command("gs://b/a b.tar", "read") == "gsutil cat 'gs://b/a b.tar'"
    with pytest.raises(ValueError):
        gopen.command("https://h/x", "write")
    with pytest.raises(ValueError):
        gopen.command("ftp2://h/x", "read")


def test_command_override(stub, monkeypatch):
    (stub / "gs" / "b").mkdir()
    (stub / "gs" / "b" / "f").write_bytes(b"abc")
    monkeypatch.setenv("JMAE_GOPEN_GS_READ", "gsutil cat {url} | tr a-z A-Z")
    assert gopen.read_bytes("gs://b/f") == b"ABC"


def test_shards_over_gs(stub):
    d = stub / "gs" / "bkt" / "imagenet-1k-wds"
    d.mkdir(parents=True)
    for k in range(2):
        _make_tar(str(d / f"train-{k}.tar"), 4, start=k * 4)
    urls = S.shard_list("gs://bkt/imagenet-1k-wds/train-{0..1}.tar")
    got = list(S.iter_samples(urls))
    assert [s["__key__"] for s in got] == [f"sample{i:05d}" for i in range(8)]
    assert got[0]["__url__"] == "gs://bkt/imagenet-1k-wds/train-0.tar"
    # the loader's dataset over the same URLs (train stream, rank split)
    _, va = create_transforms("none", 16, "none", 0.0, 0.0, 1.0)
    ds = ShardDataset("gs://bkt/imagenet-1k-wds/train-{0..1}.tar", "finetune", va, train=False, rank=0,
                      world=1, image_size=16)
    assert len(list(ds)) == 8
    # cached validation reading downloads once into the cache directory
    p = S.cached_path("gs://bkt/imagenet-1k-wds/train-1.tar", str(stub / "cache"))
    assert p.startswith(str(stub / "cache")) and os.path.getsize(p) > 0
    assert not os.path.exists("gs:")


def test_shards_over_http(stub):
    d = stub / "http" / "host" / "wds"
    d.mkdir(parents=True)
    _make_tar(str(d / "val-0.tar"), 3)
    got = list(S.iter_samples(["https://host/wds/val-0.tar"]))
    assert len(got) == 3
    with pytest.raises(Exception):
        list(S.iter_samples(["https://host/wds/missing.tar"]))


def test_checkpoint_and_pretrained_over_gs(stub):
    pre = _pre()
    pre.store.master.normal_()
    url = save_params("gs://bkt/CKPT", "pre", pre.flax_params(), "last")
    writer().flush()
    assert url == "gs://bkt/CKPT/pre-last.msgpack"
    assert (stub / "gs" / "bkt" / "CKPT" / "pre-last.msgpack").stat().st_size > 0
    assert not os.path.exists("gs:"), "a gs:// URL must not become a local directory"
    assert gopen.exists(url) and not gopen.exists("gs://bkt/CKPT/none.msgpack")
    tree = load_params(url)
    np.testing.assert_array_equal(tree["model"]["layer_0"]["ff"]["w1"]["kernel"],
                                  pre.flax_params()["model"]["layer_0"]["ff"]["w1"]["kernel"])
    vc = ViTConfig(layers=2, dim=32, heads=4, labels=10, image_size=32, patch_size=8, posemb="sincos2d",
                   layerscale=True, image_mask_ratio=None)
    ft = FinetuneModel(vc).to("cpu")
    tree = load_pretrained_params(url, ft.flax_params(), log=lambda *a: None)
    np.testing.assert_array_equal(tree["model"]["jumbo_mlp"]["w2"]["kernel"],
                                  pre.flax_params()["model"]["jumbo_mlp"]["w2"]["kernel"])


def test_write_failure_raises(stub):
    with pytest.raises(subprocess.CalledProcessError):
        write_bytes("pipe:exit 3", b"x")


def test_launcher_ckpt_dir_from_pipe_prefix(tmp_path):
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = tmp_path / "p.sh"
    script.write_text(f'source "{repo}/config/_launch.sh"\necho "CKPT=$CKPT_DIR TRAIN=$TRAIN_SHARDS"\n')
    env = dict(os.environ, NGPU="1", DATA_DIR="pipe:gsutil cat gs://bkt/data")
    env.pop("CKPT_DIR", None)
    out = subprocess.run(["bash", str(script)], env=env, capture_output=True, text=True, check=True).stdout
    assert "CKPT=gs://bkt/data/CKPT " in out
    assert "TRAIN=pipe:gsutil cat gs://bkt/data/imagenet-1k-wds/" in out
    env["DATA_DIR"] = "gs://bkt/data"
    out = subprocess.run(["bash", str(script)], env=env, capture_output=True, text=True, check=True).stdout
    assert "CKPT=gs://bkt/data/CKPT " in out


def test_pipe_output_dir_rejected():
    """A pipe: command cannot take a joined checkpoint name: the drivers refuse it as --output-dir
    and gopen.join refuses to build such a URL (the read command would swallow the bytes)."""
    import argparse

    import pytest

    from jumbo_mae_tpu_amd.train.cli import pretrain_parser
    from jumbo_mae_tpu_amd.utils import gopen

    with pytest.raises(ValueError):
        gopen.join("pipe:gsutil cat gs://b/ckpt", "run-last.msgpack")
    p = pretrain_parser()
    p.error = lambda msg: (_ for _ in ()).throw(argparse.ArgumentTypeError(msg))
    with pytest.raises(argparse.ArgumentTypeError):
        p.parse_args(["--output-dir", "pipe:cat"])
    assert p.parse_args(["--output-dir", "gs://b/out"]).output_dir == "gs://b/out"
