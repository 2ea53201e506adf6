"""Build the in-tree HIP extension ``jumbo_mae_tpu_amd/_C*.so`` for gfx950.

Direct hipcc build (no hipify, no setuptools CUDA shim): every ``*.hip`` kernel TU is compiled
with ``hipcc --offload-arch=gfx950 -O3``; the pybind/ATen glue (``bindings.cpp``) is host-only
C++ compiled with g++; the shared object is linked with hipcc against libtorch.  Objects are
cached by content hash so rebuilds only touch changed files.  Works without a GPU (cross
compile), which is what ``__graft_entry__.build()`` relies on.

Variants (``--variant``):
  release  ``_C``        the production build;
  debug    ``_C_debug``  every kernel with ``-DJM_DEBUG``: soft device checks (launch invariants
                         at kernel entry, index ranges of the MAE gathers) recorded per translation
                         unit and read back with ``debug_lines()``; selected at
                         run time with ``JMAE_EXT=debug``;
  asan     ``_C_asan``   host code (bindings + the host side of every kernel TU) built with
                         AddressSanitizer (``-Xarch_host -fsanitize=address``; bindings also UBSan; device code is
                         unchanged -- GPU ASan is not available on this pool); run python with
                         ``LD_PRELOAD=$(gcc -print-file-name=libasan.so)`` and ``JMAE_EXT=asan``.

Usage: ``python -m jumbo_mae_tpu_amd.csrc.build [--clean] [-j N] [--variant release|debug|asan]``
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

KERNELS = ["layernorm.hip", "elementwise.hip", "attention.hip", "optim.hip", "mae.hip", "gemm.hip", "gemm_tn.hip", "dropout.hip",
           "augment.hip"]


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


VARIANTS = {"release": "_C", "debug": "_C_debug", "asan": "_C_asan"}


def so_path(variant: str = "release") -> Path:
    return PKG / (VARIANTS[variant] + sysconfig.get_config_var("EXT_SUFFIX"))


def io_so_path() -> Path:
    return PKG / ("_io" + sysconfig.get_config_var("EXT_SUFFIX"))


def build_io(verbose: bool = True) -> Path:
    """Host-only pybind11 module ``_io`` (csrc/io/tario.cpp: native tar-shard reader); g++, no HIP."""
    import pybind11

    src = HERE / "io" / "tario.cpp"
    flags = ["-O2", "-fPIC", "-shared", "-std=c++17", "-pthread", "-I" + pybind11.get_include(),
             "-I" + sysconfig.get_paths()["include"], "-fvisibility=hidden"]
    BUILD.mkdir(parents=True, exist_ok=True)
    dig = _digest([src], flags)
    stamp = BUILD / f"io.{dig}.stamp"
    out = io_so_path()
    if not (out.exists() and stamp.exists()):
        tmp = str(out) + ".tmp"
        _run(["g++"] + flags + [str(src), "-o", tmp])
        os.replace(tmp, out)
        for old in BUILD.glob("io.*.stamp"):
            old.unlink()
        stamp.touch()
        if verbose:
            print(f"[jm-build] linked {out}", flush=True)
    return out


# per-file code-generation flags.  attention.hip: MFMA results in arch VGPRs instead of AGPRs --
# the attention kernels run VALU work (softmax) on every accumulator, and with the default AGPR
# form each score costs a v_accvgpr_read plus a larger register footprint (forward S=199, hd=32:
# 160 VGPR + 56 AGPR -> 109 VGPR, one occupancy step up; backward 296 -> 217).
# -fno-honor-nans: fmaxf without the NaN-quieting v_max_f32 x, x on each MFMA result (the softmax
# max is then one v_max3 per two scores).
FILE_FLAGS = {"attention.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form", "-fno-honor-nans", "-fno-slp-vectorize"]}


def build(jobs: int = 8, verbose: bool = True, clean: bool = False, variant: str = "release") -> Path:
    if clean and BUILD.exists():
        shutil.rmtree(BUILD)
    BUILD.mkdir(parents=True, exist_ok=True)
    incs, torch_lib, abi = _torch_paths()
    hdrs = sorted(HERE.glob("*.h"))
    kflags = ["--offload-arch=" + ARCH, "-O3", "-fPIC", "-std=c++17", "-I" + str(HERE),
              "-munsafe-fp-atomics", "-Wno-unused-result"]
    name = VARIANTS[variant]
    cflags = ["-O2", "-fPIC", "-std=c++17", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
              f"-D_GLIBCXX_USE_CXX11_ABI={abi}", f"-DTORCH_EXTENSION_NAME={name}", "-DTORCH_API_INCLUDE_EXTENSION_H",
              "-I" + os.path.join(ROCM, "include"), "-I" + sysconfig.get_paths()["include"]] + \
        ["-I" + p for p in incs] + ["-Wno-deprecated-declarations"]
    lflags = []
    if variant == "debug":
        kflags.append("-DJM_DEBUG=1")
        cflags.append("-DJM_DEBUG=1")
    elif variant == "asan":
        # ASan on the host side of every TU (clang, -Xarch_host) and ASan + UBSan on the g++-built
        # bindings; the runtimes are gcc's (preloaded libasan, linked libubsan)
        kflags += ["-Xarch_host", "-fsanitize=address", "-fno-omit-frame-pointer"]
        cflags += ["-fsanitize=address", "-fsanitize=undefined", "-fno-omit-frame-pointer", "-g"]
        ubsan = subprocess.run(["gcc", "-print-file-name=libubsan.so"], capture_output=True, text=True).stdout.strip()
        lflags += [ubsan]

    jobs_list = []
    for k in KERNELS:
        src = HERE / k
        if not src.exists():
            continue
        fl = kflags + FILE_FLAGS.get(k, [])
        dig = _digest([src] + hdrs, fl)
        obj = BUILD / f"{src.stem}.{dig}.o"
        jobs_list.append((obj, [HIPCC] + fl + ["-c", str(src), "-o", str(obj)]))
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
    out = so_path(variant)
    link_dig = _digest([Path(o) for o in objs], ["link", variant] + lflags)
    stamp = BUILD / f"link.{variant}.{link_dig}.stamp"
    if not (out.exists() and stamp.exists()):
        tmp = str(out) + ".tmp"
        _run([HIPCC, "-shared", "-fPIC", "--offload-arch=" + ARCH, "-o", tmp] + lflags + objs +
             ["-L" + torch_lib, "-Wl,-rpath," + torch_lib, "-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python",
              "-lc10_hip", "-ltorch_hip"])
        os.replace(tmp, out)
        for old in BUILD.glob(f"link.{variant}.*.stamp"):
            old.unlink()
        stamp.touch()
        if verbose:
            print(f"[jm-build] linked {out}", flush=True)
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("-j", type=int, default=8)
    ap.add_argument("--variant", default="release", choices=sorted(VARIANTS))
    a = ap.parse_args(argv)
    p = build(a.j, True, a.clean, a.variant)
    build_io()
    print(p)


if __name__ == "__main__":
    sys.exit(main())
