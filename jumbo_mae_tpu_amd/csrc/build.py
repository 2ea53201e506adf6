"""Build the in-tree HIP extension ``jumbo_mae_tpu_amd/_C*.so`` for gfx950.

Direct hipcc build (no hipify, no setuptools CUDA shim): every ``*.hip`` kernel TU is compiled
with ``hipcc --offload-arch=gfx950 -O3``; the pybind/ATen glue (``bindings.cpp``) is host-only
C++ compiled with g++; the shared object is linked with hipcc against libtorch.  Objects are
cached by content hash so rebuilds only touch changed files.  Works without a GPU (cross
compile), which is what ``__graft_entry__.build()`` relies on.

Usage: ``python -m jumbo_mae_tpu_amd.csrc.build [--clean] [-j N]``
"""

from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

HERE = Path(__file__).resolve().parent
PKG = HERE.parent
BUILD = PKG.parent / "build" / "jm_ext"
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")

KERNELS = ["layernorm.hip", "elementwise.hip", "attention.hip", "optim.hip", "mae.hip", "gemm.hip", "gemm_tn.hip"]


def _torch_paths():
    import torch
    from torch.utils import cpp_extension as ce

    return ce.include_paths(), os.path.join(os.path.dirname(torch.__file__), "lib"), \
        int(torch._C._GLIBCXX_USE_CXX11_ABI)


def _digest(paths, flags) -> str:
    h = hashlib.sha256()
    for p in paths:
        h.update(Path(p).read_bytes())
    h.update(" ".join(flags).encode())
    return h.hexdigest()[:16]


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("command failed:\n" + " ".join(cmd) + "\n" + r.stdout + r.stderr)
    return r


def so_path() -> Path:
    return PKG / ("_C" + sysconfig.get_config_var("EXT_SUFFIX"))


def build(jobs: int = 8, verbose: bool = True, clean: bool = False) -> Path:
    if clean and BUILD.exists():
        shutil.rmtree(BUILD)
    BUILD.mkdir(parents=True, exist_ok=True)
    incs, torch_lib, abi = _torch_paths()
    hdrs = sorted(HERE.glob("*.h"))
    kflags = ["--offload-arch=" + ARCH, "-O3", "-fPIC", "-std=c++17", "-I" + str(HERE),
              "-munsafe-fp-atomics", "-Wno-unused-result"]
    cflags = ["-O2", "-fPIC", "-std=c++17", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
              f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H",
              "-I" + os.path.join(ROCM, "include"), "-I" + sysconfig.get_paths()["include"]] + \
        ["-I" + p for p in incs] + ["-Wno-deprecated-declarations"]

    jobs_list = []
    for k in KERNELS:
        src = HERE / k
        if not src.exists():
            continue
        dig = _digest([src] + hdrs, kflags)
        obj = BUILD / f"{src.stem}.{dig}.o"
        jobs_list.append((obj, [HIPCC] + kflags + ["-c", str(src), "-o", str(obj)]))
    bsrc = HERE / "bindings.cpp"
    dig = _digest([bsrc], cflags)
    bobj = BUILD / f"bindings.{dig}.o"
    jobs_list.append((bobj, ["g++"] + cflags + ["-c", str(bsrc), "-o", str(bobj)]))

    todo = [(o, c) for o, c in jobs_list if not o.exists()]
    if verbose and todo:
        print(f"[jm-build] compiling {len(todo)} translation unit(s) for {ARCH}", flush=True)
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        futs = {ex.submit(_run, c): o for o, c in todo}
        for f in cf.as_completed(futs):
            f.result()
            if verbose:
                print(f"[jm-build]   built {futs[f].name}", flush=True)
    objs = [str(o) for o, _ in jobs_list]
    out = so_path()
    link_dig = _digest([Path(o) for o in objs], ["link"])
    stamp = BUILD / f"link.{link_dig}.stamp"
    if not (out.exists() and stamp.exists()):
        tmp = str(out) + ".tmp"
        _run([HIPCC, "-shared", "-fPIC", "--offload-arch=" + ARCH, "-o", tmp] + objs +
             ["-L" + torch_lib, "-Wl,-rpath," + torch_lib, "-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python",
              "-lc10_hip", "-ltorch_hip"])
        os.replace(tmp, out)
        for s in BUILD.glob("link.*.stamp"):
            s.unlink()
        stamp.touch()
        if verbose:
            print(f"[jm-build] linked {out}", flush=True)
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("-j", type=int, default=8)
    a = ap.parse_args(argv)
    p = build(a.j, True, a.clean)
    print(p)


if __name__ == "__main__":
    sys.exit(main())
