"""SURVEY §5 host sanitizer build: the host half of libdfu_hip (GEMM planner and tuned-table
lookup, tail-split and workspace sizing, argument validation of every entry point, error
buffer, resize taps, BN/LN sizing helpers) built with AddressSanitizer + UBSan
(`make -C dfu-multimodal_amd asan`, -Xarch_host: device code unchanged) and driven by
tests/native/host_asan.cpp on the CPU.  Passing = exit 0 and no sanitizer report."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "dfu-multimodal_amd")
BIN = os.path.join(PKG, "build_asan", "host_asan")


@pytest.mark.skipif(shutil.which("make") is None or not os.path.exists("/opt/rocm/bin/hipcc"),
                    reason="needs make and hipcc")
def test_host_logic_under_asan_ubsan():
    # the GEMM tile tables link from the normal build's objects (built first if absent)
    b = subprocess.run(["make", "-C", PKG, "-j8", "all", "asan"], capture_output=True, text=True,
                       timeout=1500)
    assert b.returncode == 0, b.stdout[-3000:] + b.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:exitcode=99",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=600, env=env)
    out = r.stdout + r.stderr
    assert "AddressSanitizer" not in out and "runtime error" not in out, out[-4000:]
    assert r.returncode == 0, out[-4000:]
    assert "all host checks passed" in r.stdout
