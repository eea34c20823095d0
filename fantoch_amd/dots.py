"""Dot = Id<ProcessId> packed into a u64 (fantoch/src/id.rs:7-62).

ProcessId (u8) in bits 56..63, sequence in bits 0..55: the packed integer
order equals the derived Ord of Id{source, sequence}.
"""
SEQ_MASK = (1 << 56) - 1


def dot(source: int, sequence: int) -> int:
    assert 0 < source < 256 and 0 <= sequence <= SEQ_MASK
    return (int(source) << 56) | int(sequence)


def dot_source(d: int) -> int:
    return int(d) >> 56


def dot_sequence(d: int) -> int:
    return int(d) & SEQ_MASK


def target_shard(d: int, n: int) -> int:
    """Dot::target_shard (fantoch/src/id.rs:58-62)."""
    return (dot_source(d) - 1) // n
