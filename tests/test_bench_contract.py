"""bench.py's roofline bookkeeping on CPU (no GPU needed): SURVEY §8(d)'s
per-command bytes, the dominant-kernel choice, and the key-order path's tile
term (B_exec + B_order: the tile kernel writes the per-key sequences,
DESIGN.md §5.1)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _probe(us, launches, alg):
    return {"avg_launch_us": us, "launches": launches, "algorithmic_bytes_per_launch": alg,
            "achieved_GBs": alg / (us * 1e-6) / 1e9, "traffic": None}


def test_sec8d_bytes_c4():
    b = bench.sec8d_bytes(1, 3, 2.04472953)
    assert b["deps"] == 84
    assert b["order"] == 16
    assert b["exec"] == pytest.approx(28.179, abs=1e-3)
    assert b["total"] == pytest.approx(184.537, abs=1e-3)


def test_roofline_dominant_kernel_and_terms():
    b8d = bench.sec8d_bytes(1, 3, 2.04472953)
    n, steps = 100_000_000, 10
    probes = {"graph_tile": _probe(5000.0, steps, 4e9), "cmd_search": _probe(3000.0, steps, 4.9e9)}
    r = bench.roofline(probes, "x", n, b8d, steps)
    assert r["kernel"] == "graph_tile"
    # command-order path: the tile kernel is the executor term alone
    assert r["algorithmic_bytes_per_step"] == pytest.approx(b8d["exec"] * n)
    assert r["achieved"] == pytest.approx(b8d["exec"] * n / 5e-3 / 1e9)
    assert r["frac"] == pytest.approx(r["achieved"] / bench.HBM_PEAK_GBS)
    # key-order path (k_ko_final ran): exec + order
    probes["ko_final"] = _probe(850.0, steps, 2.4e9)
    r = bench.roofline(probes, "x", n, b8d, steps)
    assert r["algorithmic_bytes_per_step"] == pytest.approx((b8d["exec"] + b8d["order"]) * n)
    assert "exec+order" in r["basis"]


def test_roofline_without_probes():
    r = bench.roofline({}, "graph_tile", 1, bench.sec8d_bytes(1, 3, 2.0), 1)
    assert r["frac"] == 0.0 and r["kernel"] == "graph_tile"
