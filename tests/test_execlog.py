"""Execution-log ingest (fh_execlog_*, csrc/execlog.cpp) on the CPU: the parser
needs no device.

The reference ships no execution-log fixtures, so the
format is pinned by a frame assembled byte by byte from the layouts the
reference derives (serde field order, executor/graph/executor.rs:204-222,
command.rs:11-20, deps/keys/mod.rs:18-22, id.rs:21-27) under bincode 1.3's
legacy encoding and LengthDelimitedCodec's default header (run/rw/mod.rs:
20-100) -- independently of the Python writer, which is then checked by
round trips.  Parity with a real fantoch log: unpinned (none exists here).
"""
import random

import numpy as np
import pytest

from conftest import D
from fantoch_amd import _lib as L
from fantoch_amd import execlog as E


def z(n):
    return "00" * n


# GraphExecutionInfo::Add{dot: (2,5), cmd: Command{rifl: (9,4),
# shard_to_ops: {0: {"k": Get}}, read_only: true, _empty_keys: {}},
# deps: {Dependency{dot: (1,1), shards: Some({0})}}}
HAND_ADD = "".join([
    "00000000",                  # variant 0 = Add (u32 LE)
    "02", "05" + z(7),           # dot: source u8, sequence u64
    "09" + z(7), "04" + z(7),    # rifl: client u64, sequence u64
    "01" + z(7),                 # shard_to_ops: 1 entry
    z(8),                        #   shard 0
    "01" + z(7),                 #   1 op
    "01" + z(7), "6b",           #   key "k"
    "00000000",                  #   KVOp::Get
    "01",                        # read_only = true
    z(8),                        # _empty_keys: 0 entries
    "01" + z(7),                 # deps: 1 entry
    "01", "01" + z(7),           #   dot (1,1)
    "01", "01" + z(7), z(8),     #   shards: Some({0})
])
# GraphExecutionInfo::Request{from: 3, dots: {(4,2)}}
HAND_REQ = "01000000" + "03" + z(7) + "01" + z(7) + "04" + "02" + z(7)


def framed(hexstr):
    b = bytes.fromhex(hexstr)
    return len(b).to_bytes(4, "big") + b


def test_hand_assembled_frames():
    data = framed(HAND_ADD) + framed(HAND_REQ)
    assert len(bytes.fromhex(HAND_ADD)) == 109
    lg = E.ExecLog(data, shard_id=0)
    assert lg.sizes() == (2, 2, 1, 2, 1)
    ev = lg.events()
    assert ev.kind.tolist() == [L.FH_LOG_ADD, L.FH_LOG_REQUEST]
    assert int(ev.dot[0]) == D([2, 5])
    assert (int(ev.rifl_client[0]), int(ev.rifl_seq[0])) == (9, 4)
    assert int(ev.shards[0]) == 1 and int(ev.read_only[0]) == 1
    assert ev.key_off.tolist() == [0, 1, 1] and lg.keys() == ["k"]
    assert ev.dep_off.tolist() == [0, 1, 2]
    assert [int(x) for x in ev.dep_dot] == [D([1, 1]), D([4, 2])]
    assert int(ev.dep_shards[0]) == 1
    assert int(ev.shards[1]) == 3, "a Request's shards field is the requesting shard"
    # the writer produces the same bytes
    cmd = E.encode_command((9, 4), {0: [("k", E.GET)]}, read_only=True)
    assert E.encode_add(D([2, 5]), cmd, [(D([1, 1]), [0])]).hex() == HAND_ADD
    assert E.encode_request(3, [D([4, 2])]).hex() == HAND_REQ


def test_other_shards_keys_are_not_this_shards():
    cmd = E.encode_command((1, 1), {0: [("a", (E.PUT, "v"))], 2: [("b", E.DELETE), ("c", E.DELETE)]})
    data = E.frame(E.encode_add(D([1, 1]), cmd, []))
    for shard, keys in [(0, ["a"]), (2, ["b", "c"]), (1, [])]:
        lg = E.ExecLog(data, shard_id=shard)
        ev = lg.events()
        assert lg.keys() == keys
        assert int(ev.shards[0]) == (1 << 0) | (1 << 2)


def random_log(seed, n=300):
    rng = random.Random(seed)
    frames, want = [], []
    for i in range(n):
        r = rng.random()
        if r < 0.7:
            dot = D([rng.randint(1, 9), i + 1])
            shard_ops = {s: [(f"key{rng.randrange(50)}-{j}", (E.PUT, "x" * rng.randrange(5)))
                             for j in range(rng.randint(1, 3))]
                         for s in rng.sample(range(4), rng.randint(1, 2))}
            deps = [(D([rng.randint(1, 9), rng.randint(1, 10**6)]),
                     None if rng.random() < 0.1 else rng.sample(range(4), rng.randint(1, 3)))
                    for _ in range(rng.randint(0, 5))]
            frames.append(E.encode_add(dot, E.encode_command((i, i + 7), shard_ops), deps))
            want.append(("add", dot, shard_ops, deps))
        elif r < 0.8:
            dots = [D([rng.randint(1, 9), rng.randint(1, 99)]) for _ in range(rng.randint(0, 4))]
            frames.append(E.encode_request(rng.randrange(4), dots))
            want.append(("request", dots))
        elif r < 0.9:
            dots = [D([rng.randint(1, 9), rng.randint(1, 99)]) for _ in range(rng.randint(0, 4))]
            frames.append(E.encode_executed(dots))
            want.append(("executed", dots))
        else:
            infos = [("executed", D([1, rng.randint(1, 9)])),
                     ("info", D([3, i + 1]), E.encode_command((0, 0), {1: [("q", E.GET)]}, True),
                      [(D([2, 2]), [1])])]
            frames.append(E.encode_request_reply(infos))
            want.append(("reply", infos))
    return b"".join(E.frame(f) for f in frames), want


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_round_trip_every_info_kind(seed):
    data, want = random_log(seed)
    lg = E.ExecLog(data, shard_id=0)
    ev = lg.events()
    names = lg.keys()
    e = 0
    for w in want:
        if w[0] == "add":
            _, dot, shard_ops, deps = w
            assert ev.kind[e] == L.FH_LOG_ADD and int(ev.dot[e]) == dot
            got_keys = [names[int(k)] for k in ev.key_id[ev.key_off[e]:ev.key_off[e + 1]]]
            assert got_keys == [k for k, _ in shard_ops.get(0, [])]
            assert int(ev.shards[e]) == sum(1 << s for s in shard_ops)
            got = list(zip(ev.dep_dot[ev.dep_off[e]:ev.dep_off[e + 1]].tolist(),
                           ev.dep_shards[ev.dep_off[e]:ev.dep_off[e + 1]].tolist()))
            assert got == [(d, 0 if s is None else sum(1 << x for x in set(s))) for d, s in deps]
            e += 1
        elif w[0] in ("request", "executed"):
            assert ev.kind[e] == (L.FH_LOG_REQUEST if w[0] == "request" else L.FH_LOG_EXECUTED)
            assert ev.dep_dot[ev.dep_off[e]:ev.dep_off[e + 1]].tolist() == w[1]
            e += 1
        else:
            assert ev.kind[e] == L.FH_LOG_REPLY_EXECUTED and int(ev.dot[e]) == w[1][0][1]
            assert ev.kind[e + 1] == L.FH_LOG_REPLY_INFO and int(ev.dot[e + 1]) == w[1][1][1]
            assert int(ev.read_only[e + 1]) == 1 and int(ev.shards[e + 1]) == 2
            e += 2
    assert e == len(ev.kind) == lg.sizes()[1]


def test_empty_log():
    lg = E.ExecLog(b"")
    assert lg.sizes() == (0, 0, 0, 0, 0)


@pytest.mark.parametrize("bad", [
    framed("07000000"),                          # no such GraphExecutionInfo variant
    framed(HAND_ADD)[:-1],                       # frame longer than the log
    framed(HAND_ADD + "00"),                     # trailing bytes in a frame
    framed(HAND_ADD[:-2 * 9]),                   # value truncated inside the frame
    framed(HAND_REQ.replace("04" + "02", "00" + "02")),  # dot with ProcessId 0
    b"\x00\x00",                                 # truncated frame header
])
def test_malformed_logs_are_rejected(bad):
    with pytest.raises(L.FhError) as e:
        E.ExecLog(bad)
    assert e.value.status == L.FH_EINVAL
    assert "execution log" in str(e.value)
