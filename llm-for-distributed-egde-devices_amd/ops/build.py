"""In-tree build of the edgellm HIP extension for gfx950 (MI355X).

Each ``csrc/*.hip`` kernel file is compiled by ``hipcc --offload-arch=gfx950`` into an object
(no torch headers -> fast, parallel, incremental); ``csrc/bindings.cpp`` (torch/pybind11 glue,
host-only) is compiled once; everything is linked against torch's own HIP runtime into
``ops/_C<EXT_SUFFIX>`` next to this file, so the built library travels with the repo snapshot.
Cross-compiles without a GPU.

    python -m edgellm.ops.build            # or: python llm-for-distributed-egde-devices_amd/ops/build.py
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(HERE, "..", "..", "build", "ops")
ARCH = os.environ.get("EDGELLM_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

KERNEL_FLAGS = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
                "-Wno-unused-result"]


def _torch_paths():
    import torch
    from torch.utils import cpp_extension as ce
    inc = ce.include_paths()
    lib = os.path.join(os.path.dirname(torch.__file__), "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def target_path() -> str:
    return os.path.join(HERE, "_C" + sysconfig.get_config_var("EXT_SUFFIX"))


def _stale(obj: str, deps) -> bool:
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed:\n" + " ".join(cmd) + "\n" + r.stdout)
    return r.stdout


def build(verbose: bool = False, jobs: int = 8) -> str:
    os.makedirs(BUILD, exist_ok=True)
    inc, lib, abi = _torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    header_deps = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    jobs_list = []
    objs = []
    for f in sorted(os.listdir(CSRC)):
        src = os.path.join(CSRC, f)
        if f.endswith(".hip"):
            obj = os.path.join(BUILD, f[:-4] + ".o")
            cmd = [HIPCC, *KERNEL_FLAGS, "-I", CSRC, "-c", src, "-o", obj]
        elif f.endswith(".cpp"):
            obj = os.path.join(BUILD, f[:-4] + ".o")
            cmd = [HIPCC, "-O2", "-fPIC", "-std=c++17", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
                   "-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H",
                   f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-Wno-unused-result", "-Wno-deprecated-declarations",
                   *[f"-I{p}" for p in inc], f"-I{py_inc}", "-I", CSRC, "-c", src, "-o", obj]
        else:
            continue
        objs.append(obj)
        if _stale(obj, [src] + header_deps):
            jobs_list.append(cmd)
    if jobs_list:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            for out in ex.map(_run, jobs_list):
                if verbose and out.strip():
                    print(out)
    target = target_path()
    if _stale(target, objs):
        tmp = target + ".tmp"
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", tmp,
               f"-L{lib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python",
               "-lamdhip64", f"-Wl,-rpath,{lib}"]
        _run(cmd)
        os.replace(tmp, target)          # atomic: a concurrent reader never sees a half-written library
    if verbose:
        print("built", target)
    return target


if __name__ == "__main__":
    build(verbose="-v" in sys.argv)
