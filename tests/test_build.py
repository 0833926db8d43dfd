"""The in-tree extensions build for gfx950 and load on the CPU host too.

Loading resolves every data symbol of `_C` at dlopen time, so a kernel whose
host handle the compiler failed to emit (an undefined `tdg::...` symbol)
fails here, on the CPU, instead of on the GPU box."""
import os
import subprocess

from tensorflow_distributed_on_gke_amd.ops import _ext


def test_hip_extension_loads():
    mod = _ext.C()
    assert hasattr(mod, "gemm")


def test_no_undefined_kernel_symbols():
    path = mod_path = _ext.C().__file__
    assert os.path.exists(mod_path)
    out = subprocess.run(["nm", "-D", "--undefined-only", path], capture_output=True, text=True,
                         check=True).stdout
    bad = [ln.split()[-1] for ln in out.splitlines() if "_ZN3tdg" in ln]
    assert not bad, bad[:5]
