"""The oracle's partial-replication protocol (oracle.c, restating
executor/graph/mod.rs:139-157, 168-179, 279-408 and index.rs:171-205) on the
hand-derived cases of the rules.  The reference has no unit test for these
paths; the GPU side is compared with this restatement in
lock step (tests/test_partial_exec_gpu.py)."""
from conftest import D
from oracle import oracle as O


def test_requests_first_missing_nonlocal_dependency_only():
    g = O.Graph(process_id=1, shard_id=0, n=2, f=0, shard_count=3)
    # (3,1) lives on shard 1 ((3-1)//2), (5,7) on shard 2, (2,4) is ours
    g.add_sharded(D([1, 1]), [0], [0], [(D([3, 1]), [1]), (D([5, 7]), [2, 1]), (D([2, 4]), [0, 1])])
    assert g.pending() == 1
    assert g.requests() == {1: {D([3, 1])}, 2: {D([5, 7])}}
    assert g.requests() == {}, "requests() takes the queue"
    # a second child of an already indexed missing dot: no new request
    g.add_sharded(D([1, 2]), [0], [0], [(D([3, 1]), [1]), (D([1, 1]), [0]), (D([6, 1]), [2])])
    assert g.requests() == {2: {D([6, 1])}}
    # a dependency executed when its child arrives is not missing
    g.mark_executed(D([4, 1]))
    g.add_sharded(D([1, 3]), [0], [0], [(D([4, 1]), [1]), (D([1, 2]), [0])])
    assert g.requests() == {}
    for p in ([3, 1], [5, 7], [6, 1], [2, 4]):
        g.mark_executed(D(p))
    assert g.pending() == 0
    assert g.drain()[0] == [D([1, 1]), D([1, 2]), D([1, 3])]
    assert not g.violation()


def test_process_requests_info_executed_buffered():
    g = O.Graph(process_id=2, shard_id=1, n=1, f=0, shard_count=2)
    g.add_sharded(D([2, 1]), [7], [1], [(D([2, 9]), [1]), (D([1, 5]), [0, 1])])
    g.add_sharded(D([2, 2]), [8], [1], [])
    g.handle_requests(0, [D([2, 1]), D([2, 2]), D([2, 3])])
    rep = g.request_replies()
    assert rep == {0: [("info", D([2, 1]), frozenset([1]),
                        [(D([2, 9]), frozenset([1])), (D([1, 5]), frozenset([0, 1]))]),
                       ("executed", D([2, 2]))]}
    assert g.request_replies() == {}
    g.cleanup()
    assert g.request_replies() == {}, "still unknown: stays buffered"
    g.add_sharded(D([2, 3]), [9], [1], [])
    g.cleanup()
    assert g.request_replies() == {0: [("executed", D([2, 3]))]}


def test_violations_flagged():
    g = O.Graph(process_id=1, shard_id=0, n=1, f=0, shard_count=2)
    # the requester replicates the requested command (mod.rs:313-322)
    g.add_sharded(D([1, 1]), [1], [0, 1], [(D([1, 9]), [0])])
    g.handle_requests(1, [D([1, 1])])
    assert g.violation()
    # a noop (no shard set) missing in partial replication (index.rs:190-194)
    h = O.Graph(process_id=1, shard_id=0, n=1, f=0, shard_count=2)
    h.add_sharded(D([1, 1]), [1], [0], [(D([2, 2]), None)])
    assert h.violation()
