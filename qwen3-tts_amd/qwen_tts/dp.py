"""Data-parallel serving across the GPUs of one node.

Utterances are independent, so the path shards with no data-path collective: one process per GPU,
longest-first assignment to the least-loaded rank, per-rank batched generate, host-side gather of the
results.  The only device collective is the one-time weight broadcast from rank 0 (RCCL over xGMI with
the "nccl" backend on ROCm; gloo on CPU in the tests).
"""
from __future__ import annotations

import heapq
from typing import Dict, List, Sequence

import torch
import torch.distributed as dist


def shard_longest_first(lengths: Sequence[int], world: int) -> List[List[int]]:
    """LPT schedule: items sorted by length (desc) go to the currently least-loaded rank."""
    heap = [(0, r) for r in range(world)]
    out: List[List[int]] = [[] for _ in range(world)]
    for i in sorted(range(len(lengths)), key=lambda i: (-lengths[i], i)):
        load, r = heapq.heappop(heap)
        out[r].append(i)
        heapq.heappush(heap, (load + lengths[i], r))
    return [sorted(x) for x in out]


def broadcast_weights(W: Dict[str, torch.Tensor], src: int = 0, group=None) -> None:
    """In-place broadcast of every tensor of a state dict (same names/shapes on every rank)."""
    for k in sorted(W):
        dist.broadcast(W[k], src, group=group)


def gather_results(local: list, indices: List[int], total: int, dst: int = 0, group=None):
    """Host-side gather of per-rank results back into global order on `dst` (None elsewhere)."""
    world = dist.get_world_size(group)
    payload = list(zip(indices, local))
    objs = [None] * world if dist.get_rank(group) == dst else None
    dist.gather_object(payload, objs, dst=dst, group=group)
    if objs is None:
        return None
    out = [None] * total
    for part in objs:
        for i, v in part:
            out[i] = v
    return out


def reduce_timing(dt: float, audio_seconds: float, device=None, group=None):
    """(max wall time over ranks, sum of generated audio seconds) -- the bench's whole-job numbers."""
    t = torch.tensor([dt], dtype=torch.float64, device=device)
    a = torch.tensor([audio_seconds], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    dist.all_reduce(a, op=dist.ReduceOp.SUM, group=group)
    return float(t), float(a)
