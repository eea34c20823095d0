"""Full-size parity on the GPU: the engine's outputs on the BASELINE.json
configurations against the oracle's digests (tests/golden/digests.json, made
by tests/golden/make_digests.py), and full-size properties where the
incremental oracle cannot finish (its Tarjan is quadratic on C3's stream-wide
SCC and C5's million-member SCC).  Streams are regenerated here by the seeded
counter-based generator (same library, same streams)."""
import json
import os

import numpy as np
import pytest

from fantoch_amd.engine import Engine
from fullsize import CONFIGS, check_properties, digest_deps, digest_labels, digest_perkey

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "digests.json")


def gold(name):
    with open(GOLD) as fh:
        d = json.load(fh)
    if name not in d:
        pytest.skip(f"no digest for {name} (run tests/golden/make_digests.py)")
    return d[name]


def run_engine(s):
    eng = Engine(s.key_space, n=5)
    eng.stage(s)
    eng.run()
    r = eng.results()
    eng.close()
    return r


def check_digests(g, r, what=("deps", "labels", "perkey")):
    if "deps" in what:
        assert digest_deps(r["dep_off"], r["deps"]) == g["deps"], "committed deps"
    if "labels" in what:
        assert digest_labels(r["scc_label"]) == g["labels"], "SCC partition (min-dot labels)"
    if "perkey" in what:
        assert digest_perkey(r["key_off"], r["key_seq"]) == g["perkey"], "per-key sequences"


def test_c1_full_digest():
    g = gold("c1")
    s = CONFIGS["c1"]["workload"]().generate(g["n"], logs=True, times=False)
    check_digests(g, run_engine(s))


def test_c4_full_100m_digest():
    """The bench.py headline stream at its full 100M commands."""
    g = gold("c4")
    s = CONFIGS["c4"]["workload"]().generate(g["n"], logs=True, times=False)
    check_digests(g, run_engine(s))


def test_c4_key_shard_digest():
    """Key shard 0 of 8 with global dots (the multi-GPU bench's rank 0)."""
    g = gold("c4shard")
    c = CONFIGS["c4shard"]
    s = c["workload"]().generate_shard(c["total"], c["nshards"], c["shard"])
    assert s.n == g["n"]
    check_digests(g, run_engine(s))


def test_c4_balanced_key_shard_digest():
    """Shard 0 of 8 under the balanced key map (fh_key_owners_balanced), as
    bench.py --gpus 8 gives rank 0."""
    from fantoch_amd.workload import key_owners_balanced
    g = gold("c4shard_bal")
    c = CONFIGS["c4shard_bal"]
    w = c["workload"]()
    owner = key_owners_balanced(w.key_histogram(c["total"]), c["nshards"])
    s = w.generate_shard(c["total"], c["nshards"], c["shard"], owner=owner)
    assert s.n == g["n"]
    check_digests(g, run_engine(s))


def test_c4_weighted_key_shard_digest():
    """Shard 0 of 8 under the work-weighted key map (key_owners_weighted),
    as bench.py --gpus 8 gives rank 0: the shard holding the hottest key."""
    from fantoch_amd.workload import key_owners_weighted
    g = gold("c4shard_w")
    c = CONFIGS["c4shard_w"]
    w = c["workload"]()
    owner = key_owners_weighted(w.key_histogram(c["total"]), c["nshards"])
    s = w.generate_shard(c["total"], c["nshards"], c["shard"], owner=owner)
    assert s.n == g["n"]
    check_digests(g, run_engine(s))


@pytest.mark.parametrize("name", ["c3", "c5_12m", "c5"])
def test_prefix_digest(name):
    """C3 / the unsharded 4-key stream / C5's partial replication: everything
    against the oracle on the largest prefix it finishes."""
    g = gold(name)["prefix"]
    s = CONFIGS[name]["workload"]().generate(g["n"], logs=True, times=False)
    check_digests(g, run_engine(s))


@pytest.mark.parametrize("name", ["c3", "c5_12m"])
def test_full_size_deps_and_properties(name):
    """C3 at 10M / the 4-key stream at 12.5M: committed deps bit-exact against
    the oracle's linear-time KeyDeps + QuorumDeps pass, and the SCC / order
    properties."""
    g = gold(name)
    s = CONFIGS[name]["workload"]().generate(g["n"], logs=True, times=False)
    r = run_engine(s)
    check_digests(g, r, what=("deps",))
    check_properties(s, r)


def test_c4_full_properties():
    """Independent checks of the 100M headline output (also pinned by digest)."""
    s = CONFIGS["c4"]["workload"]().generate(20_000_000, logs=True, times=False)
    check_properties(s, run_engine(s))


def test_c5_100m_partial_replication():
    """C5 at its stated size: 100M commands of 4 keys, Atlas partial
    replication over 8 key shards, all on this GPU.  Shard h's processes are
    5h+1..5h+5, a dot comes from its target shard, and every shard collects
    with its own fast quorum and arrival order; the engine stages the 40
    processes' element logs (each sees only the command's keys on its shard).
    The committed deps must equal the oracle's shard-by-shard computation
    unioned across shards (MShardCommit, atlas.rs:559-639;
    tests/fullsize.py shard_union), and the SCC partition, execution order
    and per-key sequences pass the full-size properties (scipy SCC over the
    committed deps)."""
    g = gold("c5")
    assert g.get("shards") == 8
    s = CONFIGS["c5"]["workload"]().generate(g["n"], logs=True, times=False)
    assert s.log_elem is not None and len(s.log_off) == 41
    r = run_engine(s)
    print("c5 100M: engine done", flush=True)
    assert int(r["dep_off"][-1]) == g["ndeps"], "committed dep count"
    check_digests(g, r, what=("deps",))
    print("c5 100M: deps digest ok", flush=True)
    check_properties(s, r, log=lambda m: print("c5 100M:", m, flush=True))
