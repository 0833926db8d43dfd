"""Host sanitizers over the native runtime (csrc/runtime): the reference has
no race detection at all. GPU-side AddressSanitizer /
xnack+ builds are not available on the MI355X pool, so the sanitizers cover
the host code: ThreadSanitizer on the multi-threaded batch prefetcher and
AddressSanitizer + UndefinedBehaviorSanitizer on the TensorBundle / SSTable /
CRC32C checkpoint I/O, via a standalone self-test (csrc/tests/runtime_selftest.cpp)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = [os.path.join(ROOT, "csrc", "tests", "runtime_selftest.cpp"),
       os.path.join(ROOT, "csrc", "runtime", "data_loader.cpp"),
       os.path.join(ROOT, "csrc", "runtime", "tensor_bundle.cpp")]
CXX = shutil.which("g++") or shutil.which("clang++")


def _build_run(tmp_path, flags, what):
    exe = str(tmp_path / ("selftest_" + what))
    cmd = [CXX, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-pthread", "-msse4.2",
           "-I" + os.path.join(ROOT, "csrc", "runtime")] + flags + SRC + ["-o", exe]
    b = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert b.returncode == 0, b.stderr[-3000:]
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1",
               ASAN_OPTIONS="detect_leaks=1:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([exe, str(tmp_path), what], capture_output=True, text=True, timeout=300,
                       env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-5000:]
    assert "WARNING: ThreadSanitizer" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr
    assert "runtime error:" not in r.stderr, r.stderr[-3000:]
    assert "selftest ok" in r.stdout


@pytest.mark.skipif(CXX is None, reason="no host C++ compiler")
def test_prefetcher_thread_sanitizer(tmp_path):
    _build_run(tmp_path, ["-fsanitize=thread"], "prefetch")


@pytest.mark.skipif(CXX is None, reason="no host C++ compiler")
def test_runtime_address_ub_sanitizers(tmp_path):
    _build_run(tmp_path, ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"], "all")
