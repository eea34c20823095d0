"""Key-shard partition of a command stream across GPUs.

owner(key) = key mod world.  With one key per command every command (and its
whole dependency chain, which is per key) lives on exactly one shard, so the
shards order independently: no data-path collective.  Each shard sequences its
own dots, like fantoch's per-shard DotGen for shard `rank`'s processes
(fantoch/src/util.rs:115-122: ids n*shard+1 .. n*shard+n).
"""
from __future__ import annotations

import numpy as np

from .workload import Stream, Workload


def shard_batches(w: Workload, rank: int, world: int, batch: int, nbatches: int,
                  return_index: bool = False):
    """The `rank`-th key shard of w's global single-view stream (the C2
    shape), cut into `nbatches` batches of `batch` commands.  Keys are
    renumbered to shard-local ids (key // world).  With return_index, also
    returns the global stream index of every shard command (for checking
    against the unsharded stream).  Replica-view streams (C4) are sharded on
    the device instead, with their replica logs filtered to the shard:
    `Workload.generate_shard` (fh_workload_generate_shard)."""
    assert w.keys_per_cmd == 1 and w.views == 0, \
        "single-view 1-key streams only (replica views: Workload.generate_shard)"
    out, index = [], []
    first, local_count = 0, 0
    carry_k = np.zeros(0, dtype=np.uint64)
    carry_i = np.zeros(0, dtype=np.int64)
    n = w.n
    while len(out) < nbatches:
        s = w.generate(batch * world, first=first)
        keys = s.keys[:, 0]
        mine = keys % np.uint64(world) == np.uint64(rank)
        carry_k = np.concatenate([carry_k, (keys[mine] // np.uint64(world)).astype(np.uint64)])
        carry_i = np.concatenate([carry_i, np.nonzero(mine)[0].astype(np.int64) + first])
        first += batch * world
        while len(carry_k) >= batch and len(out) < nbatches:
            kk, ii = carry_k[:batch], carry_i[:batch]
            carry_k, carry_i = carry_k[batch:], carry_i[batch:]
            idx = np.arange(local_count, local_count + batch, dtype=np.uint64)
            local_count += batch
            src = np.uint64(rank * n + 1) + idx % np.uint64(n)
            seq = idx // np.uint64(n) + np.uint64(1)
            out.append(Stream((src << np.uint64(56)) | seq, kk.reshape(-1, 1).copy(), None, None,
                              (w.key_count + world - 1) // world))
            index.append(ii)
    return (out, index) if return_index else out
