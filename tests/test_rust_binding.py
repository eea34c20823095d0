"""The fantoch_hip Rust crate (fantoch_hip/) is not compiled here (no cargo /
rustc in the image); these CPU checks keep it honest: its extern "C" block is
the generated image of include/fantoch_hip.h (same functions, same arity), and
the trait impls the north star names are present."""
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import gen_rust_ffi as G  # noqa: E402


def test_ffi_rs_is_generated_from_the_header():
    with open(G.OUT) as fh:
        assert fh.read() == G.generate(), "run python tools/gen_rust_ffi.py"


def test_every_header_function_bound_with_its_arity():
    header = {name: len(params) for _, name, params in G.prototypes(open(G.HEADER).read())}
    src = open(G.OUT).read()
    block = src[src.index('extern "C" {'):]
    rust = {}
    for m in re.finditer(r"pub fn (fh_\w+)\((.*?)\) ->", block):
        args = [a for a in m.group(2).split(",") if a.strip()]
        rust[m.group(1)] = len(args)
    assert rust == header


def test_trait_impls_present():
    src = {f: open(os.path.join(ROOT, "fantoch_hip", "src", f)).read()
           for f in os.listdir(os.path.join(ROOT, "fantoch_hip", "src"))}
    assert "impl KeyDeps for HipKeyDeps" in src["keydeps.rs"]
    assert "impl KeyDeps for HipLockedKeyDeps" in src["keydeps.rs"]
    assert "unimplemented!" not in "".join(src.values())
    ex = src["executor.rs"]
    assert "impl Executor for HipGraphExecutor" in ex
    for m in ("fn new(", "fn cleanup(", "fn monitor_pending(", "fn handle(", "fn to_clients(",
              "fn to_executors(", "fn parallel(", "fn metrics(", "fn monitor(",
              "fn set_executor_index("):
        assert m in ex, m
    assert "impl Executor for HipPredecessorsExecutor" in src["pred.rs"]
    for f in ("Cargo.toml", "build.rs"):
        assert os.path.exists(os.path.join(ROOT, "fantoch_hip", f))
