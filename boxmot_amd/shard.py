"""Sequence sharding across GPUs (one process per GPU) and the end-of-run gather.

Independent video sequences are the unit of parallelism (the reference runs one process per
sequence, boxmot/engine/val.py:389-400); frames of one sequence are strictly sequential.  So the
multi-GPU path has NO per-frame collective: each rank owns a disjoint set of sequences, and RCCL
(torch.distributed "nccl" on ROCm; "gloo" in CPU tests) is used once at the end to gather a small
fixed-size record per sequence (frames, wall time, output rows, output checksum).
"""
from __future__ import annotations

import numpy as np


def shard_sequences(frame_counts, world: int, rank: int):
    """Longest-processing-time greedy assignment of sequences to ranks.

    ``frame_counts``: per-sequence frame counts (or an int = that many equal sequences).
    Returns the sorted sequence indices owned by ``rank``; deterministic for every rank.
    """
    if isinstance(frame_counts, (int, np.integer)):
        n = int(frame_counts)
        per = -(-n // world)
        return list(range(min(n, rank * per), min(n, (rank + 1) * per)))
    fc = np.asarray(frame_counts)
    order = np.argsort(-fc, kind="stable")
    load = np.zeros(world)
    owner = np.empty(fc.size, int)
    for i in order:
        r = int(np.argmin(load))
        owner[i] = r
        load[r] += fc[i]
    return sorted(int(i) for i in np.flatnonzero(owner == rank))


def output_checksum(rows: np.ndarray) -> float:
    """Order-sensitive checksum of an output stream (ids, det_ind and boxes); rows have 8
    columns (10 for StrongSort, whose extra quality/occlusion columns are ignored)."""
    r = np.asarray(rows, np.float64)
    r = r.reshape(-1, r.shape[-1] if r.ndim == 2 else 8)
    w = np.arange(1, r.shape[0] + 1, dtype=np.float64)
    return float((r[:, 4] * w).sum() + (r[:, 7] * 0.5 * w).sum() + r[:, :4].sum() * 1e-3)


def gather_records(records: np.ndarray, dist=None, device=None, collective: bool = False
                   ) -> np.ndarray:
    """All-gather per-sequence float64 records [n_local, k] of every rank (variable n_local):
    sizes first, then padded payloads.  Returns the concatenation in rank order.  A single rank
    returns its records without a collective unless `collective` (the one-GPU test of the RCCL
    path)."""
    import torch

    rec = np.ascontiguousarray(records, np.float64)
    if dist is None or not dist.is_initialized() or (dist.get_world_size() == 1 and not collective):
        return rec
    world = dist.get_world_size()
    k = rec.shape[1]
    n = torch.tensor([rec.shape[0]], dtype=torch.int64, device=device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n)
    sizes = [int(s.item()) for s in sizes]
    pad = max(sizes) if sizes else 0
    buf = torch.zeros((pad, k), dtype=torch.float64, device=device)
    if rec.shape[0]:
        buf[: rec.shape[0]] = torch.from_numpy(rec).to(device)
    outs = [torch.zeros_like(buf) for _ in range(world)]
    dist.all_gather(outs, buf)
    return np.concatenate([o[:s].cpu().numpy() for o, s in zip(outs, sizes)], 0)
