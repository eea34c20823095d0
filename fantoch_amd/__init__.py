"""fantoch_amd -- MI355X (gfx950) batched dependency engine for fantoch.

Host-side mirror of the reference's plug-in interfaces for the dependency
hot path, backed by the HIP C ABI (include/fantoch_hip.h):

  HipKeyDeps        KeyDeps trait   (fantoch_ps/src/protocol/common/graph/deps/keys/mod.rs:37-63)
  HipGraphExecutor  Executor trait  (fantoch/src/executor/mod.rs:27-88), GraphExecutor semantics
  Engine            fused batch engine: deps + SCC + order on device
  Workload          seeded synthetic command streams (fantoch/src/client/workload.rs)
"""
from .dots import dot, dot_source, dot_sequence  # noqa: F401
from ._lib import FhError, load  # noqa: F401

__all__ = ["dot", "dot_source", "dot_sequence", "FhError", "load"]


def __getattr__(name):
    # lazy imports so that `import fantoch_amd` works before the library is built
    if name in ("HipKeyDeps", "Dependency"):
        from . import keydeps
        return getattr(keydeps, name)
    if name in ("HipGraphExecutor", "GraphExecutionInfo"):
        from . import executor
        return getattr(executor, name)
    if name == "Engine":
        from .engine import Engine
        return Engine
    if name == "Workload":
        from .workload import Workload
        return Workload
    if name == "Command":
        from .command import Command
        return Command
    raise AttributeError(name)
