"""Host AddressSanitizer run of the C ABI (SURVEY §5 sanitizers; CPU only).

tools/asan/Makefile builds libaarmvs_asan.so -- the same sources, host code instrumented
with AddressSanitizer, device code unchanged -- and tools/asan/abi_host.cpp, which drives
every host path that needs no GPU: shape validation, the workspace carve (each state
region written end to end in a heap buffer of exactly aarmvs_sweep_workspace_bytes),
argument rejection of each entry point, error strings and the profiling bookkeeping.
ASan aborts the run on an out-of-bounds access, use-after-free or leak.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc") or shutil.which("make") is None,
                    reason="needs hipcc and make")
def test_abi_host_paths_clean_under_asan():
    r = subprocess.run(["make", "-C", os.path.join(ROOT, "tools", "asan"), "-j4", "run"],
                       capture_output=True, text=True, timeout=900)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "abi_host: ok (0 failed checks)" in out
    assert "ERROR: AddressSanitizer" not in out and "ERROR: LeakSanitizer" not in out
