"""The one cross-GPU exchange of a sharded search.

Each rank holds the insertion log of its ID shard (ssa_amd_search(...,
SSA_AMD_LOG)); rank 0 gathers the logs in rank (= ID) order with a single
torch.distributed gather -- RCCL over xGMI on the GPU box ("nccl" backend),
gloo in the CPU tests -- and replays them with ssa_amd_replay, which yields
the reference's 64-bit single-thread top-k bit for bit.
"""
from __future__ import annotations


def gather_logs(log, dist, rank: int, world: int, device):
    """Gathers per-rank logs [(score, id, qid, strand, frame), ...] to rank 0.
    Returns the concatenation in rank order on rank 0, None elsewhere."""
    import torch
    rows = [[int(h[0]), int(h[1]), *(int(x) for x in (h[2:5] if len(h) >= 5 else (0, 0, 0)))] for h in log]
    t = torch.tensor(rows or [[0, 0, 0, 0, 0]], dtype=torch.int64, device=device)
    n = torch.tensor([len(rows)], dtype=torch.int64, device=device)
    lens = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(lens, n)
    lens = [int(x.item()) for x in lens]
    mx = max(max(lens), 1)
    pad = torch.zeros((mx, 5), dtype=torch.int64, device=device)
    pad[: len(rows)] = t[: len(rows)]
    bufs = [torch.zeros_like(pad) for _ in range(world)] if rank == 0 else None
    dist.gather(pad, bufs, dst=0)
    if rank != 0:
        return None
    merged = []
    for r in range(world):
        merged += [tuple(x) for x in bufs[r][: lens[r]].tolist()]
    return merged


def global_topk(log, k: int, dist, rank: int, world: int, device):
    """Exact global top-k (rank 0) from the local shard log."""
    import libssa_amd as S
    merged = gather_logs(log, dist, rank, world, device)
    return S.replay(merged, k) if rank == 0 else None
