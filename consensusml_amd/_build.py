"""In-tree build of the native extensions (no JIT cache, no hipify, gfx950 only).

* ``consensusml_amd/_C*.so``       HIP kernels (``csrc/kernels/*.hip``, hipcc --offload-arch=gfx950)
                                   + torch/pybind11 bindings (``csrc/bindings.cpp``).
* ``consensusml_amd/_runtime*.so`` host C++ runtime (``csrc/runtime/*.cpp``): data loader,
                                   checkpoint/consensus-table IO, bucket planner. Pure C++17 +
                                   pybind11, so it also loads in the CPU-only test container.

Objects are cached under ``build/`` and rebuilt only when a source or header is newer.
Usage: ``python -m consensusml_amd._build [--force] [--only C|runtime]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import shlex
import subprocess
import sys
import sysconfig
from typing import List

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "consensusml_amd")
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(ROOT, "build", "obj")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CXX = os.environ.get("CXX", "g++")
EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _torch_paths():
    import torch  # noqa: F401  (only for include / lib paths)
    from torch.utils import cpp_extension as ce
    tdir = os.path.dirname(torch.__file__)
    return ce.include_paths(), os.path.join(tdir, "lib"), bool(torch._C._GLIBCXX_USE_CXX11_ABI)


def _pybind_include() -> str:
    import pybind11
    return pybind11.get_include()


def _newer(target: str, deps: List[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def _run(cmd: List[str], verbose: bool) -> None:
    if verbose:
        print("  $", " ".join(shlex.quote(c) for c in cmd), flush=True)
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout)
        raise RuntimeError(f"build step failed ({r.returncode}): {cmd[0]} ... {cmd[-1]}")


def _headers(d: str) -> List[str]:
    return glob.glob(os.path.join(d, "**", "*.h"), recursive=True)


def ext_path(name: str) -> str:
    return os.path.join(PKG, name + EXT_SUFFIX)


def build_kernels(force: bool = False, verbose: bool = False) -> str:
    """Compile csrc/kernels/*.hip + csrc/bindings.cpp into consensusml_amd/_C.so."""
    os.makedirs(BUILD, exist_ok=True)
    tinc, tlib, abi = _torch_paths()
    hdrs = _headers(os.path.join(CSRC, "kernels"))
    py_inc = sysconfig.get_paths()["include"]
    common = ["-O3", "-std=c++17", "-fPIC", f"-D_GLIBCXX_USE_CXX11_ABI={int(abi)}"]
    jobs = []
    objs = []
    for src in sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip"))):
        obj = os.path.join(BUILD, os.path.basename(src) + ".o")
        objs.append(obj)
        if force or _newer(obj, [src] + hdrs):
            jobs.append([HIPCC, f"--offload-arch={ARCH}", *common, "-I", CSRC, "-c", src, "-o", obj])
    bsrc = os.path.join(CSRC, "bindings.cpp")
    bobj = os.path.join(BUILD, "bindings.cpp.o")
    objs.append(bobj)
    if force or _newer(bobj, [bsrc] + hdrs):
        inc = sum((["-I", p] for p in tinc), [])
        jobs.append([HIPCC, f"--offload-arch={ARCH}", *common, "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
                     "-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H",
                     *inc, "-I", py_inc, "-I", CSRC, "-c", bsrc, "-o", bobj])
    with cf.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 4)) as ex:
        list(ex.map(lambda c: _run(c, verbose), jobs))
    out = ext_path("_C")
    if force or jobs or _newer(out, objs):
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", out,
              "-L", tlib, "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
              "-ltorch_python", f"-Wl,-rpath,{tlib}"], verbose)
    return out


def build_runtime(force: bool = False, verbose: bool = False) -> str:
    """Compile csrc/runtime/*.cpp (host C++ runtime, no HIP) into consensusml_amd/_runtime.so."""
    os.makedirs(BUILD, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    if not srcs:
        return ""
    hdrs = _headers(os.path.join(CSRC, "runtime"))
    py_inc = sysconfig.get_paths()["include"]
    flags = ["-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-pthread", "-Wall",
             "-I", _pybind_include(), "-I", py_inc, "-I", CSRC]
    jobs, objs = [], []
    for src in srcs:
        obj = os.path.join(BUILD, "rt_" + os.path.basename(src) + ".o")
        objs.append(obj)
        if force or _newer(obj, [src] + hdrs):
            jobs.append([CXX, *flags, "-c", src, "-o", obj])
    with cf.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 4)) as ex:
        list(ex.map(lambda c: _run(c, verbose), jobs))
    out = ext_path("_runtime")
    if force or jobs or _newer(out, objs):
        _run([CXX, "-shared", "-fPIC", "-pthread", *objs, "-o", out], verbose)
    return out


def build(force: bool = False, verbose: bool = False, only: str = "") -> None:
    if only in ("", "runtime"):
        p = build_runtime(force, verbose)
        if verbose and p:
            print("built", p)
    if only in ("", "C"):
        p = build_kernels(force, verbose)
        if verbose:
            print("built", p)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--only", choices=["C", "runtime"], default="")
    ap.add_argument("-q", "--quiet", action="store_true")
    a = ap.parse_args()
    build(a.force, not a.quiet, a.only)


if __name__ == "__main__":
    main()
