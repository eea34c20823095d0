"""CPU-side checks of the C-ABI library: it loads, exports every symbol that
include/fantoch_hip.h declares, and its host-only parts (workload generator)
behave.  No compute on a device here."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from conftest import ROOT
from fantoch_amd import _lib as L
from fantoch_amd.workload import Workload

HEADER = os.path.join(ROOT, "include", "fantoch_hip.h")


def declared_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"\b(fh_[a-z0-9_]+)\s*\(", txt)))


def test_library_loads_and_exports_every_declared_symbol():
    lib = L.load()
    syms = declared_symbols()
    assert len(syms) >= 25
    for s in syms:
        assert hasattr(lib, s), s
        assert s in L.SIGNATURES, f"{s} missing from the ctypes signature table"


def test_version_and_errors():
    lib = L.load()
    assert b"gfx950" in lib.fh_version()
    st = lib.fh_keydeps_create(0, None, None)
    assert st == L.FH_EINVAL
    assert b"null" in lib.fh_last_error()


def test_workload_deterministic_and_in_range():
    w = Workload.zipf(0.99, 1 << 16, k=2, views=3, window=64)
    a = w.generate(5000)
    b = w.generate(1000, first=2000)
    assert np.array_equal(a.dots[2000:3000], b.dots)
    assert np.array_equal(a.keys[2000:3000], b.keys)
    assert np.array_equal(a.fq_time[2000:3000], b.fq_time)
    assert a.keys.max() < a.key_space
    assert np.all(a.keys[:, 0] != a.keys[:, 1])  # unique keys per command
    # dots: process 1 + i mod n, sequence i / n + 1 (DotGen)
    i = np.arange(5000, dtype=np.uint64)
    assert np.array_equal(a.dots >> np.uint64(56), 1 + i % np.uint64(5))
    assert np.array_equal(a.dots & np.uint64((1 << 56) - 1), i // np.uint64(5) + np.uint64(1))
    # coordinator arrives at its submission slot; members within the window
    assert np.array_equal(a.fq_time[:, 0], i * np.uint64(64))
    assert np.all(a.fq_time[:, 1:] >= a.fq_time[:, :1])
    assert np.all(a.fq_time[:, 1:] < (i[:, None] + np.uint64(64)) * np.uint64(64))


def test_workload_rejects_reference_invalid_configs():
    # workload.rs:39-48: ConflictRate 100% with more than one key panics
    with pytest.raises(L.FhError):
        Workload.conflict_rate_(100, k=2).generate(10)


def test_zipf_is_skewed_like_the_zipf_crate():
    s = Workload.zipf(0.99, 1 << 20).generate(200_000)
    u, c = np.unique(s.keys, return_counts=True)
    # rank 1 (id 0) is the most frequent; P(rank 1) = 1/H_{K,s}
    K, sexp = 1 << 20, 0.99
    H = np.sum(np.arange(1, K + 1, dtype=np.float64) ** -sexp)
    p0 = c[u == 0][0] / len(s.keys)
    assert abs(p0 - 1 / H) < 0.01


def test_small_pass_wait_has_a_deadline():
    """graph_small's host wait (graph_small.h poll_completion) against a
    stream that never completes: FH_EHIP with fh_last_error set after the
    deadline, instead of spinning (no GPU involved)."""
    import time
    lib = L.load()
    t0 = time.perf_counter()
    st = lib.fh_selftest_poll_deadline(50)
    dt = time.perf_counter() - t0
    assert st == L.FH_EHIP
    assert b"did not complete within 50 ms" in lib.fh_last_error()
    assert 0.04 < dt < 5.0
    assert lib.fh_selftest_poll_deadline(0) == L.FH_EINVAL
