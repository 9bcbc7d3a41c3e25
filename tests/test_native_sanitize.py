"""The host half of the C ABI built with AddressSanitizer + UBSan (sanitizers
on host code) and driven by a native C++ caller against the C oracle (tests/native/).
CPU only: ans_capi.cpp and ans_core.hpp need no HIP."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None or shutil.which("gcc") is None, reason="needs gcc/g++")
def test_host_abi_under_asan_ubsan(tmp_path):
    san = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]
    obj = tmp_path / "oracle.o"
    subprocess.check_call(["gcc", "-std=c11", *san, "-c", os.path.join(ROOT, "oracle", "ans_oracle.c"), "-o", str(obj)])
    exe = tmp_path / "abi_sanitize"
    subprocess.check_call(["g++", "-std=c++17", *san, "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "native", "abi_sanitize.cpp"),
                           os.path.join(ROOT, "shuffle-coding_amd", "csrc", "ans_capi.cpp"), str(obj), "-o", str(exe)])
    # verify_asan_link_order=0: the environment may preload a library ahead of the ASan runtime
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    out = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=300)
    assert out.returncode == 0, out.stderr[-4000:]
    assert "abi_sanitize ok" in out.stdout
