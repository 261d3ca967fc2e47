"""Host C++ runtime (crc32c, TFRecord, TensorBundle, CIFAR prefetch ring) under AddressSanitizer +
UndefinedBehaviorSanitizer and ThreadSanitizer.  The self-test executable links
the runtime sources directly, so no sanitizer runtime has to be preloaded into Python.  GPU code is
not sanitized here (no GPU ASan / xnack+ on this pool); kernels are checked by the numerics tests."""
import glob
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RT = os.path.join(ROOT, "csrc", "runtime")


def _build_and_run(tmp_path, flags, env_extra):
    cxx = shutil.which("g++") or shutil.which("clang++")
    if cxx is None:
        pytest.skip("no host C++ compiler")
    exe = str(tmp_path / "selftest")
    srcs = sorted(glob.glob(os.path.join(RT, "*.cpp"))) + [os.path.join(RT, "tests", "runtime_selftest.cpp")]
    cmd = [cxx, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-pthread"] + flags + srcs + ["-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0 and "sanitizer" in r.stderr.lower() and "cannot find" in r.stderr.lower():
        pytest.skip("sanitizer runtime not installed: " + r.stderr[-300:])
    assert r.returncode == 0, r.stderr[-3000:]
    env = dict(os.environ, **env_extra)
    out = subprocess.run([exe, str(tmp_path)], capture_output=True, text=True, env=env, timeout=300)
    assert out.returncode == 0 and "runtime selftest OK" in out.stdout, (out.stdout + out.stderr)[-4000:]


def test_runtime_asan_ubsan(tmp_path):
    _build_and_run(tmp_path, ["-fsanitize=address,undefined", "-fno-sanitize-recover=all"],
                   {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0:halt_on_error=1"})


def test_runtime_tsan(tmp_path):
    _build_and_run(tmp_path, ["-fsanitize=thread"], {"TSAN_OPTIONS": "halt_on_error=1:second_deadlock_stack=1"})
