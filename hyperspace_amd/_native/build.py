"""Builds the native libraries in-tree (no JIT cache, so the .so files travel with the repo
snapshot to the GPU box):

* ``libhs_kernels.so`` — HIP/CDNA4 kernels for gfx950 (``csrc/kernels/*.hip``), compiled with
  ``hipcc --offload-arch=gfx950``; C ABI launchers called through ctypes.
* ``libhs_runtime.so`` — host C++ runtime (``csrc/runtime/*.cpp``): hipRTC whole-stage codegen
  (compile, code-object cache, module launch) and roctx pipeline-stage markers.  Host-only C++
  against the HIP runtime, built with hipcc.
* ``_hs_host*.so`` — CPython extension for the query front end's host hot paths
  (``csrc/host/hs_host.cpp``), built with g++.

Usage: ``python -m hyperspace_amd._native.build [--force]``.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
CSRC = os.path.join(ROOT, "csrc")
KERNEL_LIB = os.path.join(HERE, "libhs_kernels.so")
RUNTIME_LIB = os.path.join(HERE, "libhs_runtime.so")
ARCH = os.environ.get("HS_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


def _newer(target: str, sources) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in sources)


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return r


def build_kernels(force: bool = False) -> str:
    kdir = os.path.join(CSRC, "kernels")
    srcs = sorted(os.path.join(kdir, f) for f in os.listdir(kdir) if f.endswith(".hip"))
    hdrs = [os.path.join(kdir, f) for f in os.listdir(kdir) if f.endswith(".h")]
    if not force and not _newer(KERNEL_LIB, srcs + hdrs):
        return KERNEL_LIB
    objdir = os.path.join(HERE, "obj")
    os.makedirs(objdir, exist_ok=True)
    hipcc = _hipcc()

    def compile_one(src):
        obj = os.path.join(objdir, os.path.basename(src) + ".o")
        if force or _newer(obj, [src] + hdrs):
            _run([hipcc, f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-c", src,
                  "-o", obj, "-Wno-unused-result", "-munsafe-fp-atomics"])
        return obj

    with cf.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(compile_one, srcs))
    tmp = KERNEL_LIB + ".tmp"
    _run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs)
    os.replace(tmp, KERNEL_LIB)
    return KERNEL_LIB


def build_runtime(force: bool = False) -> str:
    rdir = os.path.join(CSRC, "runtime")
    if not os.path.isdir(rdir):
        return ""
    srcs = sorted(os.path.join(rdir, f) for f in os.listdir(rdir) if f.endswith(".cpp"))
    hdrs = [os.path.join(rdir, f) for f in os.listdir(rdir) if f.endswith(".h")]
    if not srcs:
        return ""
    if not force and not _newer(RUNTIME_LIB, srcs + hdrs):
        return RUNTIME_LIB
    tmp = RUNTIME_LIB + ".tmp"
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    # host-only C++ against the HIP runtime + hipRTC (whole-stage codegen); hipcc supplies the
    # platform defines and include paths
    _run([_hipcc(), "-O3", "-std=c++17", "-fPIC", "-shared", "-pthread", "-o", tmp] + srcs +
         [f"-L{rocm}/lib", "-lhiprtc", "-lamdhip64", "-ldl", "-lz", f"-Wl,-rpath,{rocm}/lib"])
    os.replace(tmp, RUNTIME_LIB)
    return RUNTIME_LIB


def host_ext_path() -> str:
    import sysconfig
    return os.path.join(HERE, "_hs_host" + (sysconfig.get_config_var("EXT_SUFFIX") or ".so"))


def build_host(force: bool = False) -> str:
    """``_hs_host``: CPython extension for the query front end's host hot paths
    (``csrc/host/hs_host.cpp``: the plan cache's fingerprint walk), plain g++."""
    import sysconfig
    src = os.path.join(CSRC, "host", "hs_host.cpp")
    out = host_ext_path()
    if not os.path.exists(src):
        return ""
    if not force and not _newer(out, [src]):
        return out
    cxx = os.environ.get("CXX") or shutil.which("g++") or "c++"
    tmp = out + ".tmp"
    _run([cxx, "-O2", "-std=c++17", "-fPIC", "-shared", "-fno-strict-aliasing",
          f"-I{sysconfig.get_paths()['include']}", src, "-o", tmp])
    os.replace(tmp, out)
    return out


def build_all(force: bool = False):
    build_host(force)
    return build_kernels(force), build_runtime(force)


if __name__ == "__main__":
    print(build_all("--force" in sys.argv))
