#!/usr/bin/env python3
"""Build the in-tree HIP extension ``theroundtaible_amd/_C*.so`` for gfx950 with hipcc.

Explicit hipcc lines (no hipify, no CUDA compatibility layer, no JIT cache in ~/.cache):
every ``csrc/*.hip`` is compiled as HIP device+host code for ``--offload-arch=gfx950``;
``bindings.cpp`` is compiled as host C++ against the torch headers; the shared object
links against *torch's* bundled HIP runtime (same SONAME as /opt/rocm's) so one HIP
runtime is loaded per process. Incremental: objects are rebuilt only when a source or
header is newer. Works on a CPU-only machine (hipcc cross-compiles).
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
PKG = os.path.join(ROOT, "theroundtaible_amd")
BUILD = os.path.join(ROOT, "build", "csrc")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# per-file flags: no SLP packing of f32 VALU beside MFMAs (v_pk_mul_f32 costs more issue cycles
# than two scalar ops there; MI355X_MICROARCH "price of one filler beside MFMAs")
FILE_FLAGS = {"attention_prefill32.hip": ["-fno-slp-vectorize"]}


def torch_paths():
    import torch
    from torch.utils.cpp_extension import include_paths, library_paths
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return include_paths(), library_paths()[0], abi


def ext_path() -> str:
    return os.path.join(PKG, "_C" + sysconfig.get_config_var("EXT_SUFFIX"))


def _newer(src: str, obj: str, deps) -> bool:
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(p) > t for p in [src] + list(deps))


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return r.stderr


def build(verbose: bool = False, jobs: int = 8) -> str:
    os.makedirs(BUILD, exist_ok=True)
    incs, torch_lib, abi = torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    headers = glob.glob(os.path.join(HERE, "*.h"))
    common = ["-O3", "-fPIC", "-std=c++17", f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-D__HIP_PLATFORM_AMD__=1",
              "-DUSE_ROCM=1", "-Wno-unused-result", "-Wno-deprecated-declarations", "-Wno-unused-command-line-argument"]
    jobs_list = []
    objs = []
    for src in sorted(glob.glob(os.path.join(HERE, "*.hip"))):
        obj = os.path.join(BUILD, os.path.basename(src) + ".o")
        objs.append(obj)
        if _newer(src, obj, headers):
            jobs_list.append([HIPCC, "-x", "hip", f"--offload-arch={ARCH}", "-munsafe-fp-atomics", *common,
                              *FILE_FLAGS.get(os.path.basename(src), []), "-I", HERE, "-c", src, "-o", obj])
    bsrc = os.path.join(HERE, "bindings.cpp")
    bobj = os.path.join(BUILD, "bindings.cpp.o")
    objs.append(bobj)
    if _newer(bsrc, bobj, []):
        jobs_list.append([HIPCC, *common, "-I", py_inc, *sum((["-I", i] for i in incs), []),
                          "-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H", "-c", bsrc, "-o", bobj])
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        for err in ex.map(_run, jobs_list):
            if verbose and err.strip():
                print(err)
    out = ext_path()
    if jobs_list or not os.path.exists(out):
        link = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", out, f"-L{torch_lib}",
                "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python", "-lamdhip64",
                f"-Wl,-rpath,{torch_lib}"]
        _run(link)
    return out


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv))
