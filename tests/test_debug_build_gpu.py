"""Debug build (``_C_debug``, -DJM_DEBUG): the soft device checks are wired end to end and the
flagship ViT-L/16 pretraining step (every kernel at its headline shapes) violates none of them.

Runs in a child process with ``JMAE_EXT=debug`` so the release extension of this process is not
replaced."""

import os
import subprocess
import sys
import textwrap

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = textwrap.dedent("""
    import torch
    from jumbo_mae_tpu_amd.ops import _ext
    ext = _ext.load(True)
    assert ext.__name__.endswith("_C_debug") and ext.debug_build
    assert ext.debug_lines() == {}
    ext.debug_selftest(0)
    assert ext.debug_lines() == {}
    ext.debug_selftest(1)                      # deliberately failing check
    lines = ext.debug_lines()
    assert set(lines) == {"elementwise"} and lines["elementwise"] > 0, lines
    assert ext.debug_lines() == {}             # reading cleared it

    from jumbo_mae_tpu_amd.config import decoder_config, vit_config
    from jumbo_mae_tpu_amd.models.mae import PretrainModel
    from jumbo_mae_tpu_amd.optim.flat import FlatOptimizer
    from jumbo_mae_tpu_amd.optim.schedule import warmup_cosine_decay_schedule
    from jumbo_mae_tpu_amd.train.engine import Trainer
    from jumbo_mae_tpu_amd.utils.rng import RngStreams
    sched = warmup_cosine_decay_schedule(1e-6, 1e-3, 2, 10, 1e-5)
    vc = vit_config("vit_large_patch16", labels=0, posemb="sincos2d")
    m = PretrainModel(vc, decoder_config()).to("cuda", torch.bfloat16, seed=0)
    opt = FlatOptimizer(m.store, "adamw", sched, b2=0.95, weight_decay=0.05, num_layers=vc.layers)
    tr = Trainer(m, opt, None, RngStreams({}, 0, "cuda"))
    imgs = torch.randint(0, 256, (16, 3, 224, 224), dtype=torch.uint8, device="cuda")
    for _ in range(2):
        loss = tr.train_step([(imgs,)])["loss"]
    torch.cuda.synchronize()
    assert torch.isfinite(loss)
    _ext.debug_check()
    print("DEBUG_BUILD_OK", float(loss))
""")


def test_debug_build_checks_clean_on_flagship_step():
    so = [f for f in os.listdir(os.path.join(ROOT, "jumbo_mae_tpu_amd")) if f.startswith("_C_debug")]
    if not so:
        pytest.fail("debug extension not built: python -m jumbo_mae_tpu_amd.csrc.build --variant debug")
    env = dict(os.environ, JMAE_EXT="debug", PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    r = subprocess.run([sys.executable, "-c", SCRIPT], capture_output=True, text=True, timeout=110, env=env, cwd=ROOT)
    assert r.returncode == 0 and "DEBUG_BUILD_OK" in r.stdout, (r.stdout[-3000:], r.stderr[-3000:])
