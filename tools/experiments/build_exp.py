#!/usr/bin/env python3
"""Build the EXPERIMENT extension ``tools/experiments/_exp*.so`` (gfx950, hipcc).

Kernels here were measured and not adopted (profiles/experiments/): the persistent decode
layer (decode_layer.hip), the loader-wave LDS-ring GEMM (ring_gemm.hip) and the MALL prefetch
(prefetch.hip). They are kept reproducible but out of the product extension
(``theroundtaible_amd._C``); their tests live next to them and are not collected by
``pytest tests/``. Reuses csrc/build.py's flags and the csrc/ headers.

    python tools/experiments/build_exp.py && python -m pytest tools/experiments -m gpu
"""
from __future__ import annotations

import glob
import os
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
CSRC = os.path.join(ROOT, "csrc")
sys.path.insert(0, CSRC)
import build as csrc_build  # noqa: E402

BUILD = os.path.join(ROOT, "build", "experiments")


def ext_path() -> str:
    return os.path.join(HERE, "_exp" + sysconfig.get_config_var("EXT_SUFFIX"))


def build() -> str:
    os.makedirs(BUILD, exist_ok=True)
    incs, torch_lib, abi = csrc_build.torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    common = ["-O3", "-fPIC", "-std=c++17", f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-D__HIP_PLATFORM_AMD__=1",
              "-DUSE_ROCM=1", "-Wno-unused-result", "-Wno-deprecated-declarations"]
    objs = []
    for src in sorted(glob.glob(os.path.join(HERE, "*.hip"))):
        obj = os.path.join(BUILD, os.path.basename(src) + ".o")
        subprocess.run([csrc_build.HIPCC, "-x", "hip", f"--offload-arch={csrc_build.ARCH}", "-munsafe-fp-atomics",
                        *common, "-I", CSRC, "-c", src, "-o", obj], check=True)
        objs.append(obj)
    bobj = os.path.join(BUILD, "exp_bindings.cpp.o")
    subprocess.run([csrc_build.HIPCC, *common, "-I", py_inc, *sum((["-I", i] for i in incs), []),
                    "-DTORCH_EXTENSION_NAME=_exp", "-DTORCH_API_INCLUDE_EXTENSION_H", "-c",
                    os.path.join(HERE, "exp_bindings.cpp"), "-o", bobj], check=True)
    objs.append(bobj)
    out = ext_path()
    subprocess.run([csrc_build.HIPCC, "-shared", "-fPIC", f"--offload-arch={csrc_build.ARCH}", *objs, "-o", out,
                    f"-L{torch_lib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python",
                    "-lamdhip64", f"-Wl,-rpath,{torch_lib}"], check=True)
    return out


def load():
    """The experiment module (import torch first; raises if not built)."""
    import torch  # noqa: F401
    sys.path.insert(0, HERE)
    import _exp  # type: ignore
    return _exp


if __name__ == "__main__":
    print(build())
