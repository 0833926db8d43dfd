"""In-tree native build (no JIT cache, no hipify): generates a ninja file that
compiles every HIP kernel for gfx950 with hipcc, the torch binding unit, and
the pure-C++ host runtime, and links

  tensorflow_distributed_on_gke_amd/_C.so       (HIP kernels + torch bindings)
  tensorflow_distributed_on_gke_amd/_native.so  (TensorBundle I/O, CRC32C, data loader)

The .so files are git-ignored but live in the package directory, so they travel
with the repository snapshot to the GPU box. `python -m
tensorflow_distributed_on_gke_amd.build` (or __graft_entry__.build()) runs it;
the build is incremental.
"""
from __future__ import annotations

import os
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
PKG = Path(__file__).resolve().parent
CSRC = ROOT / "csrc"
BUILD = ROOT / "build"
ARCH = os.environ.get("TDG_OFFLOAD_ARCH", "gfx950")

HIP_SOURCES = sorted((CSRC / "kernels").glob("*.hip"))
BINDING = CSRC / "bindings.cpp"
NATIVE_SOURCES = sorted((CSRC / "runtime").glob("*.cpp"))


def _torch_paths():
    import torch
    from torch.utils import cpp_extension as ce

    inc = ce.include_paths(device_type="cuda")
    lib = str(Path(torch.__file__).parent / "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _pybind_include():
    import pybind11

    return pybind11.get_include()


def write_ninja() -> Path:
    BUILD.mkdir(exist_ok=True)
    inc, tlib, abi = _torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    hipcc = f"{rocm}/bin/hipcc"
    incs = " ".join(f"-I{p}" for p in inc)
    hip_flags = (
        f"-fPIC -O3 -std=c++17 --offload-arch={ARCH} -I{CSRC}/include "
        "-Wno-unused-result -ffp-contract=fast"
    )
    bind_flags = (
        f"-fPIC -O2 -std=c++17 -x c++ -D__HIP_PLATFORM_AMD__=1 -DUSE_ROCM=1 "
        f"-DTORCH_EXTENSION_NAME=_C -DTORCH_API_INCLUDE_EXTENSION_H "
        f"-D_GLIBCXX_USE_CXX11_ABI={abi} -I{CSRC}/include {incs} -I{py_inc} -I{rocm}/include "
        "-Wno-deprecated-declarations"
    )
    native_flags = (
        f"-fPIC -O3 -std=c++17 -msse4.2 -I{CSRC}/runtime -I{_pybind_include()} -I{py_inc} "
        f"-D_GLIBCXX_USE_CXX11_ABI={abi}"
    )
    torch_libs = (
        f"-L{tlib} -lc10 -lc10_hip -ltorch -ltorch_cpu -ltorch_hip -ltorch_python "
        f"-Wl,-rpath,{tlib}"
    )
    lines = [
        "ninja_required_version = 1.3",
        f"hipcc = {hipcc}",
        f"hip_flags = {hip_flags}",
        f"bind_flags = {bind_flags}",
        f"native_flags = {native_flags}",
        "rule hip",
        "  command = $hipcc $hip_flags -MD -MF $out.d -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = HIPCC $in",
        "rule bind",
        "  command = $hipcc $bind_flags -MD -MF $out.d -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = BIND $in",
        "rule cxx",
        "  command = g++ $native_flags -MD -MF $out.d -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = CXX $in",
        "rule link_hip",
        f"  command = $hipcc -shared -fPIC $in -o $out {torch_libs}",
        "  description = LINK $out",
        "rule link_cxx",
        "  command = g++ -shared -fPIC $in -o $out -lpthread",
        "  description = LINK $out",
    ]
    objs = []
    for s in HIP_SOURCES:
        o = BUILD / (s.stem + ".hip.o")
        lines.append(f"build {o}: hip {s}")
        objs.append(str(o))
    ob = BUILD / "bindings.o"
    lines.append(f"build {ob}: bind {BINDING}")
    objs.append(str(ob))
    ext = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    lines.append(f"build {PKG / ('_C' + ext)}: link_hip {' '.join(objs)}")
    nobjs = []
    for s in NATIVE_SOURCES:
        o = BUILD / (s.stem + ".o")
        lines.append(f"build {o}: cxx {s}")
        nobjs.append(str(o))
    lines.append(f"build {PKG / ('_native' + ext)}: link_cxx {' '.join(nobjs)}")
    nf = BUILD / "build.ninja"
    text = "\n".join(lines) + "\n"
    if not nf.exists() or nf.read_text() != text:
        nf.write_text(text)
    return nf


def build(verbose: bool = False, jobs: int | None = None) -> None:
    nf = write_ninja()
    j = jobs or min(16, os.cpu_count() or 4)
    cmd = ["ninja", "-f", str(nf), f"-j{j}"]
    if verbose:
        cmd.append("-v")
    r = subprocess.run(cmd, cwd=str(ROOT), capture_output=not verbose, text=True)
    if r.returncode != 0:
        msg = (r.stdout or "") + (r.stderr or "")
        raise RuntimeError(f"native build failed:\n{msg[-8000:]}")


if __name__ == "__main__":
    build(verbose="-v" in sys.argv)
    print("built:", ", ".join(p.name for p in PKG.glob("_*.so")))
