"""bench.py's data-parallel flow end to end on 2 gloo ranks (CPU): the exact code the driver's
multi-GPU scaling run executes under torchrun -- rank/world from the env, broadcast init, bucketed
reducer overlapped with the backward, per-bucket optimizer ranges, timing max over ranks, one JSON
line from rank 0 -- with the RCCL backend swapped for gloo and a tiny model."""

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


@pytest.mark.parametrize("extra", [[], ["--reduce-dtype", "bf16", "--grad-accum", "2"], ["--no-overlap"],
                                   ["--shard-optimizer"]])
def test_bench_two_ranks_cpu(extra):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--cpu", "--model", "vit_tiny_patch16",
           "--batch-per-gpu", "4", "--image-size", "64", "--bucket-mb", "0.5"] + extra
    env = dict(os.environ, OMP_NUM_THREADS="2")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd="/tmp", env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2"
    assert out["config"]["global_batch"] == 8 and out["steps"] == 2 and out["warmup"] == 1
    assert out["value"] > 0 and out["ms_per_step"] > 0
    assert out["replica_weight_checksum_spread"] == 0.0  # replicas bit-identical after the steps
    assert out["config"]["final_loss"] == out["config"]["final_loss"]  # not NaN
    if "--grad-accum" in extra:
        assert out["config"]["grad_accum"] == 2
    # self-calibration of the first multi-GPU run: one timed collective per distinct bucket size of
    # the real plan (what tools/dp_exposure_model.py --sweep reads) and the traced step's bucket
    # readiness times
    sweep = out["collective_sweep"]
    esz = 2 if "bf16" in extra else 4
    plan = {sp["bytes"] for sp in out["dp_ready_spans"] if not sp["partial"]}
    assert len(sweep) == len(plan)  # one row per distinct bucket size (rounded to world elements)
    assert all(min(abs(r["bytes"] - b) for b in plan) < 2 * esz for r in sweep)
    key = "reduce_scatter_busbw_GBs" if "--shard-optimizer" in extra else "allreduce_busbw_GBs"
    assert sweep and all(r[key] > 0 and r["world"] == 2 and r["bytes"] % esz == 0 for r in sweep)
    spans = out["dp_ready_spans"]
    assert spans and all(0 <= sp["ready_ms"] <= out["dp_traced_step_ms"] for sp in spans)
    assert out["reducer"]["mode"] == ("zero1-reduce-scatter" if "--shard-optimizer" in extra else "all-reduce")
