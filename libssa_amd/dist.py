"""The one cross-GPU exchange of a sharded search, over
torch.distributed -- the fallback beside the library's own RCCL gather
(ssa_amd_gather_logs, csrc/dist.cpp), with the same shape.

Each rank holds the insertion log of its ID shard (ssa_amd_search(...,
SSA_AMD_LOG)); rank 0 gathers the logs in rank (= ID) order with a single
gather of fixed-size slots to rank 0 -- RCCL over xGMI on the GPU box ("nccl"
backend), gloo in the CPU tests -- and replays them with ssa_amd_replay, which
yields the reference's 64-bit single-thread top-k bit for bit.  A log longer
than its slot sends the rest of its rows to rank 0 point to point.
"""
from __future__ import annotations


# rows per rank of the single fixed-size exchange; a shard log is a few
# dozen to a few hundred entries (k * (1 + ln(shard / k)) expected), longer
# ones send their remainder point to point
LOG_CAP = 512


def _rows(log):
    return [[int(h[0]), int(h[1]), *(int(x) for x in (h[2:5] if len(h) >= 5 else (0, 0, 0)))] for h in log]


def gather_logs(log, dist, rank: int, world: int, device, cap: int = LOG_CAP):
    """Gathers per-rank logs [(score, id, qid, strand, frame), ...] to rank 0.
    Returns the concatenation in rank order on rank 0, None elsewhere.

    One gather of a fixed [cap + 1, 5] int64 slot per rank to rank 0 (row 0
    holds the log length) -- a single collective per search.  A rank whose log
    exceeds cap sends the remaining rows to rank 0 (dist.send), which knows
    from the slot headers whom to receive from (dist.recv); no other rank
    takes part."""
    import torch
    rows = _rows(log)
    n = len(rows)
    buf = torch.zeros((cap + 1, 5), dtype=torch.int64, device=device)
    buf[0, 0] = n
    if n:
        buf[1:min(n, cap) + 1] = torch.tensor(rows[:cap], dtype=torch.int64, device=device)
    bufs = [torch.empty_like(buf) for _ in range(world)] if rank == 0 else None
    dist.gather(buf, bufs, dst=0)
    if rank != 0:
        if n > cap:
            dist.send(torch.tensor(rows[cap:], dtype=torch.int64, device=device), dst=0)
        return None
    lens = [int(b[0, 0]) for b in bufs]
    merged = []
    for r in range(world):
        if r == 0:
            merged += [tuple(x) for x in rows]
            continue
        merged += [tuple(x) for x in bufs[r][1:min(lens[r], cap) + 1].tolist()]
        if lens[r] > cap:
            rest = torch.empty((lens[r] - cap, 5), dtype=torch.int64, device=device)
            dist.recv(rest, src=r)
            merged += [tuple(x) for x in rest.tolist()]
    return merged


def global_topk(log, k: int, dist, rank: int, world: int, device, cap: int = LOG_CAP):
    """Exact global top-k (rank 0) from the local shard log."""
    import libssa_amd as S
    merged = gather_logs(log, dist, rank, world, device, cap)
    return S.replay(merged, k) if rank == 0 else None
