#!/usr/bin/env python3
"""Native build driver for tensorflow_examples_amd.

Builds two in-tree shared libraries (they travel to the GPU box with the repo
snapshot; nothing is installed into site-packages):

* ``tensorflow_examples_amd/_lib/libtfx_ops.so`` -- every hand-written HIP
  kernel (``csrc/kernels/*.hip``, compiled for gfx950 only) plus the
  ``TORCH_LIBRARY(tfx, ...)`` registrations (``csrc/torch_ops/*.cpp``).
  Loaded with ``torch.ops.load_library`` by ``tensorflow_examples_amd.ops``.
* ``tensorflow_examples_amd/_lib/libtfx_rt.so`` -- the host runtime that the
  reference gets from TF's C++ core: parameter-server service (replaces TF's
  gRPC master/worker services), CRC32C + TFRecord/tfevents writer (replaces
  TF's EventsWriter), IDX reader.  Plain C ABI, loaded with ctypes, no torch.

No hipify, no CUDA shims: the sources are HIP/C++ for CDNA4 directly.
Incremental: an object is rebuilt when its source or any header is newer.

Usage: ``python build.py [--jobs N] [--force] [--only ops|rt] [--asan]``
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(ROOT, "csrc")
OUT = os.path.join(ROOT, "tensorflow_examples_amd", "_lib")
OBJ = os.path.join(ROOT, "build", "obj")
ARCH = os.environ.get("TFX_OFFLOAD_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")


def _torch_paths():
    import torch  # noqa: F401  (only for paths / ABI flag)
    tdir = os.path.dirname(torch.__file__)
    inc = [os.path.join(tdir, "include"),
           os.path.join(tdir, "include", "torch", "csrc", "api", "include"),
           sysconfig.get_paths()["include"]]
    lib = os.path.join(tdir, "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _newer(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed:\n" + " ".join(cmd) + "\n" + r.stdout + r.stderr)
    return r.stderr


def build_ops(jobs, force, extra_flags=()):
    inc, tlib, abi = _torch_paths()
    headers = glob.glob(os.path.join(CSRC, "include", "*.h")) + glob.glob(os.path.join(CSRC, "kernels", "*.h"))
    kern = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    bind = sorted(glob.glob(os.path.join(CSRC, "torch_ops", "*.cpp")))
    os.makedirs(OBJ, exist_ok=True)
    os.makedirs(OUT, exist_ok=True)
    common = ["-O3", "-fPIC", "-std=c++17", f"-I{os.path.join(CSRC, 'include')}",
              "-D__HIP_PLATFORM_AMD__=1", "-Wno-unused-result", *extra_flags]
    jobs_list = []
    for s in kern:
        o = os.path.join(OBJ, os.path.basename(s) + ".o")
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-c", s, "-o", o, *common,
               "-munsafe-fp-atomics"]
        jobs_list.append((s, o, cmd))
    for s in bind:
        o = os.path.join(OBJ, os.path.basename(s) + ".o")
        cmd = [HIPCC, "-c", s, "-o", o, *common, f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
               "-DUSE_ROCM=1", "-DTORCH_EXTENSION_NAME=tfx_ops", *[f"-I{p}" for p in inc]]
        jobs_list.append((s, o, cmd))
    todo = [(s, o, c) for s, o, c in jobs_list if force or _newer(o, [s, *headers])]
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        for fut in [ex.submit(_run, c) for _, _, c in todo]:
            fut.result()
    so = os.path.join(OUT, "libtfx_ops.so")
    objs = [o for _, o, _ in jobs_list]
    if force or todo or _newer(so, objs):
        _run([HIPCC, "-shared", f"--offload-arch={ARCH}", "-o", so, *objs, f"-L{tlib}",
              "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-lamdhip64",
              f"-Wl,-rpath,{tlib}"])
    return so


def build_rt(jobs, force, extra_flags=()):
    srcs = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    headers = glob.glob(os.path.join(CSRC, "runtime", "*.h")) + glob.glob(os.path.join(CSRC, "include", "*.h"))
    os.makedirs(OBJ, exist_ok=True)
    os.makedirs(OUT, exist_ok=True)
    cxx = shutil.which("g++") or "c++"
    flags = ["-O2", "-fPIC", "-std=c++17", "-pthread", "-Wall", f"-I{os.path.join(CSRC, 'include')}",
             *extra_flags]
    if "-fsanitize" not in " ".join(extra_flags):
        flags.append("-msse4.2")
    objs, todo = [], []
    for s in srcs:
        o = os.path.join(OBJ, "rt_" + os.path.basename(s) + ".o")
        objs.append(o)
        if force or _newer(o, [s, *headers]):
            todo.append([cxx, "-c", s, "-o", o, *flags])
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        for fut in [ex.submit(_run, c) for c in todo]:
            fut.result()
    so = os.path.join(OUT, "libtfx_rt.so")
    if force or todo or _newer(so, objs):
        _run([cxx, "-shared", "-o", so, *objs, "-pthread", *extra_flags])
    return so


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--only", choices=["ops", "rt"], default=None)
    ap.add_argument("--asan", action="store_true", help="host-only ASAN build of the runtime lib")
    a = ap.parse_args(argv)
    out = []
    if a.only in (None, "rt"):
        extra = ("-fsanitize=address", "-fno-omit-frame-pointer", "-g") if a.asan else ()
        out.append(build_rt(a.jobs, a.force, extra))
    if a.only in (None, "ops"):
        out.append(build_ops(a.jobs, a.force))
    for p in out:
        print("built", os.path.relpath(p, ROOT))


if __name__ == "__main__":
    sys.exit(main())
