"""Host-side AddressSanitizer run of the extension's argument validation (``_C_asan``: bindings
under ASan + UBSan, kernel TUs' host code under ASan; device code unchanged -- GPU ASan is not
available on this pool).  Every binding is called with CPU tensors / bad shapes and must reject
them with a Python exception, with no sanitizer report.  Skipped unless the variant was built:
``python -m jumbo_mae_tpu_amd.csrc.build --variant asan``."""

import os
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = textwrap.dedent("""
    import torch
    from jumbo_mae_tpu_amd.ops import _ext
    ext = _ext.load(True)
    assert ext.__name__.endswith("_C_asan")
    x = torch.randn(4, 8, 32)
    b16 = torch.randn(64, 64).bfloat16()
    calls = {
        "layernorm_fwd": lambda: ext.layernorm_fwd(x, torch.ones(32), torch.zeros(32), 1e-6, torch.bfloat16),
        "gemm_nt": lambda: ext.gemm_nt(b16, b16),
        "gemm_tn_wgrad": lambda: ext.gemm_tn_wgrad(b16, b16, torch.zeros(64, 64)),
        "gelu_fwd": lambda: ext.gelu_fwd(b16),
        "colsum": lambda: ext.colsum(b16, torch.zeros(64)),
    }
    rejected = 0
    for name, fn in calls.items():
        try:
            fn()
        except (RuntimeError, TypeError, ValueError) as e:
            rejected += 1
    assert rejected == len(calls), rejected
    assert ext.debug_lines() == {}
    print("ASAN_HOST_OK", rejected)
""")


def _lib(name):
    return subprocess.run(["gcc", f"-print-file-name={name}"], capture_output=True, text=True).stdout.strip()


def test_bindings_validation_under_asan():
    if not any(f.startswith("_C_asan") for f in os.listdir(os.path.join(ROOT, "jumbo_mae_tpu_amd"))):
        pytest.skip("ASan variant not built (python -m jumbo_mae_tpu_amd.csrc.build --variant asan)")
    asan, std = _lib("libasan.so"), _lib("libstdc++.so")
    if not os.path.exists(asan):
        pytest.skip("libasan not available")
    env = dict(os.environ, JMAE_EXT="asan", LD_PRELOAD=f"{asan} {std}", ASAN_OPTIONS="detect_leaks=0",
               PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    r = subprocess.run([sys.executable, "-c", SCRIPT], capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0 and "ASAN_HOST_OK" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error:" not in r.stderr, r.stderr[-4000:]
