import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")


def load_golden(name):
    with open(os.path.join(GOLDEN, name)) as fh:
        return json.load(fh)


def D(pair):
    """[source, sequence] -> packed dot (fantoch/src/id.rs:21-27 order)."""
    return (int(pair[0]) << 56) | int(pair[1])


def UD(dot):
    return [dot >> 56, dot & ((1 << 56) - 1)]


class Interner:
    """Key = String (fantoch/src/kvs.rs:6) -> dense u64 id, as the shim does."""

    def __init__(self):
        self.ids = {}

    def __call__(self, key):
        if key not in self.ids:
            self.ids[key] = len(self.ids)
        return self.ids[key]

    def many(self, keys):
        return [self(k) for k in keys]


@pytest.fixture
def golden():
    return load_golden


@pytest.fixture(scope="session", autouse=True)
def _torch_hip_runtime_first(request):
    """torch's wheel bundles its own HIP + HSA runtime (torch/lib), the
    library links /opt/rocm's; in one process the second runtime to
    initialise sees no GPU if it is torch's ("No HIP GPUs are available",
    measured on the GPU box), so a session with GPU tests brings torch's up
    first.  Only the torch-plumbing tests (device tensors, RCCL) need it."""
    if any(it.get_closest_marker("gpu") for it in request.session.items):
        import torch
        if torch.cuda.is_available():
            torch.zeros(1, device="cuda")
    yield
