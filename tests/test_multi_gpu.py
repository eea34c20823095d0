"""fh_multi_*: key shards on several engines (here: several engines on the one
GPU of the box, devices [0, 0, 0]) compose to the single engine's outputs on
the same stream, and to the oracle's."""
import numpy as np
import pytest

from fantoch_amd.engine import Engine
from fantoch_amd.multi import MultiEngine
from fantoch_amd.workload import Workload
from fullsize import check_properties
from test_engine_gpu import oracle_pipeline

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("ndev", [2, 3])
def test_multi_shards_match_single_engine_and_oracle(ndev):
    w = Workload.zipf(0.99, 1 << 14, k=1, views=3, window=64, seed=41)
    s = w.generate(60_000, logs=True)
    one = Engine(s.key_space, n=5)
    one.stage(s)
    one.run()
    r1 = one.results()
    m = MultiEngine(s.key_space, [0] * ndev, n=5)
    m.stage(s)
    assert sum(m.shard_sizes()) == s.n
    m.run()
    r = m.results()
    for k in ("dep_off", "deps", "scc_label", "key_off", "key_seq"):
        assert np.array_equal(r[k], r1[k]), k
    dep_off, deps, ex, lab, kso, ks = oracle_pipeline(s)
    assert np.array_equal(r["deps"], deps) and np.array_equal(r["key_seq"], ks)
    check_properties(s, r)
    # rewind + rerun is identical
    m.rewind()
    m.run()
    r2 = m.results()
    for k in r:
        assert np.array_equal(r[k], r2[k]), k


def test_multi_rejects_multi_key_streams():
    from fantoch_amd import _lib as L
    s = Workload.zipf(0.99, 1 << 10, k=2, views=3, window=64, seed=3).generate(1000, logs=True)
    m = MultiEngine(s.key_space, [0, 0])
    with pytest.raises(L.FhError):
        m.stage(s)


def test_multi_failed_staging_leaves_nothing_to_run():
    """A staging that fails validation (a key id >= key_space) drops the
    previous staging: run() and results() refuse instead of combining the new
    partition with the old engines."""
    from fantoch_amd import _lib as L
    w = Workload.zipf(0.99, 1 << 10, k=1, views=3, window=64, seed=5)
    s = w.generate(5000, logs=True)
    m = MultiEngine(s.key_space, [0, 0])
    m.stage(s)
    m.run()
    assert len(m.results()["deps"]) > 0
    bad = w.generate(7000, logs=True)
    bad.keys[123, 0] = np.uint64(s.key_space)  # out of the key space
    with pytest.raises(L.FhError):
        m.stage(bad)
    with pytest.raises(L.FhError):
        m.results()
    with pytest.raises(L.FhError):
        m.run()
    # a good staging afterwards works again (the next commands of the
    # stream: the engines' command logs keep the first batch's dots)
    s2 = w.generate(5000, first=5000, logs=True)
    m.stage(s2)
    m.run()
    assert len(m.results()["deps"]) > 0
