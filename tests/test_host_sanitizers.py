"""The C++ host runtime (csrc/host) under AddressSanitizer + UndefinedBehaviorSanitizer.

Host code only: the self-test driver and ckpt_io.cpp are compiled together with
``-fsanitize=address,undefined`` and run as a plain executable (no Python, no GPU), so every
heap/stack overflow, use-after-free, leak or UB in the checkpoint I/O and the CPU AdamW fails
the test with the sanitizer report.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_host_runtime_asan_ubsan(tmp_path):
    exe = str(tmp_path / "host_selftest")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=all", "-fopenmp", "-mavx2", "-mfma", "-msse4.2",
           os.path.join(ROOT, "tests", "native", "host_runtime_test.cpp"),
           os.path.join(ROOT, "csrc", "host", "ckpt_io.cpp"), "-o", exe, "-lpthread", "-lz"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    # verify_asan_link_order=0: the environment may preload its own (non-allocator) library first
    env = {**os.environ, "ASAN_OPTIONS": "detect_leaks=1:halt_on_error=1:verify_asan_link_order=0",
           "UBSAN_OPTIONS": "print_stacktrace=1:halt_on_error=1", "OMP_NUM_THREADS": "4"}
    r = subprocess.run([exe, str(tmp_path)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "self-test OK" in r.stdout


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
@pytest.mark.parametrize("san", ["address,undefined", "thread"])
def test_aio_engine_sanitizers(tmp_path, san):
    """The NVMe AIO engine (csrc/host/aio.cpp) under ASan+UBSan and under ThreadSanitizer (race detection
    on the submit / worker / wait / destroy paths)."""
    exe = str(tmp_path / "aio_selftest")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", f"-fsanitize={san}",
           "-fno-sanitize-recover=all", os.path.join(ROOT, "tests", "native", "aio_test.cpp"),
           os.path.join(ROOT, "csrc", "host", "aio.cpp"), "-o", exe, "-lpthread"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    env = {**os.environ, "ASAN_OPTIONS": "detect_leaks=1:halt_on_error=1:verify_asan_link_order=0",
           "UBSAN_OPTIONS": "print_stacktrace=1:halt_on_error=1", "TSAN_OPTIONS": "halt_on_error=1"}
    r = subprocess.run([exe, str(tmp_path)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "aio self-test OK" in r.stdout
