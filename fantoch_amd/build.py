"""Builds fantoch_amd/libfantoch_hip.so (hipcc, gfx950) in-tree.

Usage: python -m fantoch_amd.build [--force] [-j N]
Objects go to build/ (git-ignored); the shared library is written next to this
file so that it travels with the repository snapshot to the GPU box.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(ROOT, "build", "obj")
LIB = os.path.join(HERE, "libfantoch_hip.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"

COMMON = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function",
          f"-I{os.path.join(ROOT, 'include')}", f"-I{CSRC}"]


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))


def headers():
    return sorted(glob.glob(os.path.join(CSRC, "*.h")) +
                  glob.glob(os.path.join(ROOT, "include", "*.h")))


def _newest(paths):
    return max((os.path.getmtime(p) for p in paths), default=0.0)


def _compile(src: str, force: bool) -> str:
    obj = os.path.join(OBJ, os.path.basename(src) + ".o")
    if not force and os.path.exists(obj) and os.path.getmtime(obj) >= max(
            os.path.getmtime(src), _newest(headers())):
        return obj
    cmd = [HIPCC, *COMMON, "-c", src, "-o", obj]
    if src.endswith(".hip"):
        cmd[1:1] = ["-x", "hip", f"--offload-arch={ARCH}"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj


def build(force: bool = False, jobs: int = 8, verbose: bool = False) -> str:
    os.makedirs(OBJ, exist_ok=True)
    srcs = sources()
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        objs = list(ex.map(lambda s: _compile(s, force), srcs))
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < _newest(objs):
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", LIB, *objs,
               "-lpthread"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    if verbose:
        print(f"built {LIB}")
    return LIB


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=min(16, os.cpu_count() or 4))
    a = ap.parse_args(argv)
    build(a.force, a.j, verbose=True)


if __name__ == "__main__":
    sys.exit(main())
