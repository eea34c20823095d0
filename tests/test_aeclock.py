"""The executed clock (AEClock, fantoch_amd/csrc/dotindex.h): host-only
differential test against a plain set of dots (tests/aeclock_check.cpp).

AEClock<ProcessId> (threshold crate; graph/mod.rs:50,91-95, tarjan.rs:133-135,
296): a contiguous frontier per process plus exceptions.  The library keeps
exceptions near the frontier as per-process bit rings and the rest in a hash
set, and takes an executor pass's executed dots in one bulk add; this checks
add / add_all / raise_frontier / contains / exceptions on random streams that
cross the ring's 4,096-sequence window.  No GPU: the clock is host code (the
harness is compiled with hipcc for the header's HIP includes, host only).
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_aeclock_matches_a_set(tmp_path):
    exe = tmp_path / "aeclock_check"
    src = os.path.join(ROOT, "tests", "aeclock_check.cpp")
    inc = os.path.join(ROOT, "fantoch_amd", "csrc")
    subprocess.run([HIPCC, "-O1", "-std=c++17", "-I", inc, src, "-o", str(exe)], check=True,
                   capture_output=True, timeout=240)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stdout + r.stderr
