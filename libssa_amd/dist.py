"""The one cross-GPU exchange of a sharded search.

Each rank holds the insertion log of its ID shard (ssa_amd_search(...,
SSA_AMD_LOG)); rank 0 gathers the logs in rank (= ID) order with a single
torch.distributed all_gather of fixed-size buffers -- RCCL over xGMI on the GPU box ("nccl" backend),
gloo in the CPU tests -- and replays them with ssa_amd_replay, which yields
the reference's 64-bit single-thread top-k bit for bit.
"""
from __future__ import annotations


# rows per rank of the single fixed-size exchange; a shard log is a few
# dozen to a few hundred entries (k * (1 + ln(shard / k)) expected), longer
# ones take the two-step variable-size path
LOG_CAP = 512


def _rows(log):
    return [[int(h[0]), int(h[1]), *(int(x) for x in (h[2:5] if len(h) >= 5 else (0, 0, 0)))] for h in log]


def gather_logs(log, dist, rank: int, world: int, device, cap: int = LOG_CAP):
    """Gathers per-rank logs [(score, id, qid, strand, frame), ...] to rank 0.
    Returns the concatenation in rank order on rank 0, None elsewhere.

    One all_gather of a fixed [cap + 1, 5] int64 buffer per rank (row 0 holds
    the log length) -- a single RCCL collective per search.  If any rank's
    log exceeds cap, every rank sees it in the headers and they fall back to
    an exact-size gather."""
    import torch
    rows = _rows(log)
    n = len(rows)
    buf = torch.zeros((cap + 1, 5), dtype=torch.int64, device=device)
    buf[0, 0] = n
    if 0 < n <= cap:
        buf[1:n + 1] = torch.tensor(rows, dtype=torch.int64, device=device)
    bufs = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(bufs, buf)
    lens = torch.stack([b[0, 0] for b in bufs]).tolist()
    if max(lens) <= cap:
        if rank != 0:
            return None
        parts = [bufs[r][1:lens[r] + 1] for r in range(world) if lens[r] > 0]
        return [tuple(x) for x in torch.cat(parts).tolist()] if parts else []
    # rare: some log is longer than cap -- gather exact sizes
    mx = max(lens)
    pad = torch.zeros((mx, 5), dtype=torch.int64, device=device)
    if n:
        pad[:n] = torch.tensor(rows, dtype=torch.int64, device=device)
    out = [torch.zeros_like(pad) for _ in range(world)] if rank == 0 else None
    dist.gather(pad, out, dst=0)
    if rank != 0:
        return None
    merged = []
    for r in range(world):
        merged += [tuple(x) for x in out[r][: lens[r]].tolist()]
    return merged


def global_topk(log, k: int, dist, rank: int, world: int, device, cap: int = LOG_CAP):
    """Exact global top-k (rank 0) from the local shard log."""
    import libssa_amd as S
    merged = gather_logs(log, dist, rank, world, device, cap)
    return S.replay(merged, k) if rank == 0 else None
