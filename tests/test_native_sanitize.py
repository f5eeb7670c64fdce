"""Host-side sanitizer run of the native C++ runtime: the runtime and a
randomized self-test are compiled with AddressSanitizer + UndefinedBehaviorSanitizer and run."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_runtime_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "runtime_selftest")
    srcs = [os.path.join(ROOT, "csrc", "runtime", "runtime.cpp"),
            os.path.join(ROOT, "csrc", "tests", "runtime_selftest.cpp")]
    cmd = ["g++", "-O1", "-g", "-std=c++17", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
           "-fno-sanitize-recover=all", "-o", exe] + srcs
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "runtime selftest OK" in r.stdout
