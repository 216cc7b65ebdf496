"""xfshard.py — how a batch and its counters split across ranks (host logic).

The multi-GPU model: packets are independent, so a batch
splits into contiguous per-rank ranges; rule tables are replicated with
identical slot indices; per-rule hits and per-action stats are sums over
ranks, exactly like the reference's per-CPU values summed at readout
(xdp-filter/xdp-filter.c:93-103).  xfg_comm_allreduce() does the device-side
sum over RCCL; these helpers state the same arithmetic for the host and the
CPU tests.
"""
import numpy as np

COUNTER_SHIFT = 6
FLAG_MASK = (1 << COUNTER_SHIFT) - 1


def shard_range(n: int, world: int, rank: int):
    """Contiguous [start, start + count) of rank `rank` out of `world`;
    the first n % world ranks take one extra packet."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, extra = divmod(n, world)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def split_hits(vals: np.ndarray):
    """Reference values (hits << 6 | flags) -> (hits, flags)."""
    v = np.asarray(vals, np.uint64)
    return v >> np.uint64(COUNTER_SHIFT), v & np.uint64(FLAG_MASK)


def reduced_values(per_rank_vals):
    """Values after the all-reduce as each rank reads them: its own flags,
    hits summed over ranks (xfg_comm_allreduce semantics)."""
    hits = sum(split_hits(v)[0] for v in per_rank_vals)
    return [(hits << np.uint64(COUNTER_SHIFT)) | split_hits(v)[1] for v in per_rank_vals]
