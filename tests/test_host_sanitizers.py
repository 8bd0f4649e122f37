"""Host-code sanitizers: the C++ host runtime
(ops/csrc/host/fedmx_host.cpp — CSV reader, exact AUC) built with
AddressSanitizer + UndefinedBehaviorSanitizer (+ a ThreadSanitizer build for
the multi-threaded CSV path) and driven by tests/native/host_sanitize_driver.cpp
as a standalone executable.  CPU only; GPU-side sanitizers are not available
on the MI355X pool."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "fedmse_decentralized_amd", "ops", "csrc", "host", "fedmx_host.cpp")
DRIVER = os.path.join(ROOT, "tests", "native", "host_sanitize_driver.cpp")


def _cxx():
    for c in ("g++", "clang++"):
        if shutil.which(c):
            return c
    pytest.skip("no host C++ compiler")


def _build_and_run(tmp_path, flags, env_extra):
    exe = str(tmp_path / "driver")
    cmd = [_cxx(), "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", *flags, SRC, DRIVER, "-o", exe, "-pthread"]
    b = subprocess.run(cmd, capture_output=True, text=True)
    if b.returncode != 0 and "sanitize" in b.stderr:
        pytest.skip(f"sanitizer runtime unavailable: {b.stderr[-300:]}")
    assert b.returncode == 0, b.stderr
    env = dict(os.environ)
    env.pop("LD_PRELOAD", None)  # the sanitizer runtime must come first in the process
    env.update(env_extra)
    scratch = tmp_path / "scratch"
    scratch.mkdir()
    r = subprocess.run([exe, str(scratch)], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "all checks passed" in r.stdout


def test_host_runtime_asan_ubsan(tmp_path):
    _build_and_run(tmp_path, ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"],
                   {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0:halt_on_error=1"})


def test_host_runtime_tsan(tmp_path):
    _build_and_run(tmp_path, ["-fsanitize=thread"], {"TSAN_OPTIONS": "halt_on_error=1"})
