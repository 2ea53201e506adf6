"""The data-parallel path on a real RCCL communicator, on a one-GPU box.

``JMAE_FORCE_PG=1`` makes bench.py create the process group and the bucketed ``GradReducer`` even
at world size 1 (parallel/dist.py ``forced_group``).  Under torchrun with one rank that runs every
RCCL line the driver's multi-GPU scaling run executes -- ``init_process_group("nccl",
device_id=...)``, async ``all_reduce(AVG)`` per bucket issued during the backward, the per-bucket
optimizer ranges queued behind each reduction, device barriers, the max-over-ranks timing -- and
since AVG over one rank is the identity, the result must equal the plain single-process step bit
for bit.  The CPU twin (gloo, ``--cpu``) runs in the default suite.
Reference: the pmap/pmean step of /root/reference/src/pretraining.py:125-159."""

import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(args, torchrun: bool, force: bool, timeout: int = 300):
    bench = [os.path.join(ROOT, "bench.py")] + args
    if torchrun:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
               "--master-addr", "127.0.0.1", "--master-port", str(_port())] + bench
    else:
        cmd = [sys.executable] + bench
    env = dict(os.environ, OMP_NUM_THREADS="2", JMAE_FORCE_PG="1" if force else "0")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd="/tmp", env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def _check_equal(args):
    plain = _run(args, torchrun=False, force=False)
    dp = _run(args, torchrun=True, force=True)
    assert plain.get("reducer") is None
    if "reducer" in dp:
        assert dp["reducer"] is not None and dp["reducer"]["buckets"] >= 2, dp
    assert dp["config"]["final_loss"] == plain["config"]["final_loss"], (dp, plain)
    if "weight_checksum" in plain:
        # a few GPU reductions (LayerNorm / bias parameter partials) add with float atomics, so two
        # runs may differ in the last bit of some weights: a few ulps of the fp64 checksum (1.2e-12
        # relative seen on one box), far below any real divergence
        assert abs(dp["weight_checksum"] - plain["weight_checksum"]) <= 1e-11 * plain["weight_checksum"], (dp, plain)
    return plain, dp


PRETRAIN = ["--gpus", "1", "--steps", "2", "--warmup", "1", "--model", "vit_tiny_patch16",
            "--batch-per-gpu", "32", "--bucket-mb", "0.5"]


def test_forced_group_matches_plain_cpu():
    _check_equal(PRETRAIN[:-4] + ["--batch-per-gpu", "4", "--image-size", "64", "--bucket-mb", "0.5", "--cpu"])


@pytest.mark.gpu
def test_rccl_pretrain_matches_plain():
    _check_equal(PRETRAIN)


@pytest.mark.gpu
def test_rccl_pretrain_bf16_reduce_and_accum():
    out = _run(PRETRAIN + ["--reduce-dtype", "bf16", "--grad-accum", "2"], torchrun=True, force=True)
    assert out["config"]["final_loss"] == out["config"]["final_loss"] and out["reducer"] is not None


@pytest.mark.gpu
def test_rccl_finetune_matches_plain():
    _check_equal(["--task", "finetune", "--gpus", "1", "--steps", "2", "--warmup", "1", "--model",
                  "vit_tiny_patch16", "--batch-per-gpu", "32", "--bucket-mb", "0.5"])


@pytest.mark.gpu
def test_rccl_finetune_accum_matches_plain():
    """Classifier bench at a per-GPU batch above --max-micro-batch: accumulated micro-steps."""
    plain, dp = _check_equal(["--task", "finetune", "--gpus", "1", "--steps", "2", "--warmup", "1", "--model",
                              "vit_tiny_patch16", "--batch-per-gpu", "32", "--max-micro-batch", "16",
                              "--bucket-mb", "0.5"])
    assert dp["config"]["grad_accum"] == 2 and dp["config"]["micro_batch"] == 16, dp["config"]


def test_forced_group_zero1_matches_plain_cpu():
    _check_equal(PRETRAIN[:-4] + ["--batch-per-gpu", "4", "--image-size", "64", "--bucket-mb", "0.5", "--cpu",
                                  "--shard-optimizer"])


@pytest.mark.gpu
def test_rccl_pretrain_zero1_matches_plain():
    """ZeRO-1 on a 1-rank RCCL communicator: reduce_scatter_tensor / all_gather_into_tensor in
    place on the flat buffers, the sharded AdamW rows and the shadow re-cast all execute; over one
    rank they are identities, so the step must equal the plain one."""
    plain, dp = _check_equal(PRETRAIN + ["--shard-optimizer"])
    assert dp["reducer"]["mode"] == "zero1-reduce-scatter", dp


@pytest.mark.gpu
def test_rccl_linear_zero1_lars_matches_plain():
    """LARS (per-leaf trust ratios: the sharded norms are all-reduced) on the linear-probe step."""
    _check_equal(["--task", "linear", "--gpus", "1", "--steps", "2", "--warmup", "1", "--batch-per-gpu", "32",
                  "--bucket-mb", "0.5", "--shard-optimizer"])
