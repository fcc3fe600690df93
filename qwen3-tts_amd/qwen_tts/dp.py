"""Data-parallel serving across the GPUs of one node.

Utterances are independent, so the path shards with no data-path collective: one process per GPU,
longest-first assignment to the least-loaded rank, per-rank continuous-batching decode, host-side gather of the
results.  The only device collective is the one-time weight broadcast from rank 0 (RCCL over xGMI with
the "nccl" backend on ROCm; gloo on CPU in the tests), coalesced into a few large flat buffers.
"""
from __future__ import annotations

import heapq
from typing import Dict, List, Optional, Sequence

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


def broadcast_weights(W: Dict[str, torch.Tensor], src: int = 0, group=None, bucket_bytes: int = 1 << 30) -> int:
    """In-place broadcast of a state dict (same names / shapes / dtypes on every rank), coalesced: tensors of one
    dtype are packed in name order into flat buckets of <= bucket_bytes and each bucket is one collective (a few
    calls of ~1 GiB instead of one per tensor: xGMI ring broadcasts are bandwidth-bound per link, so large messages
    run at link speed while hundreds of small ones pay the per-call latency).  src is a GLOBAL rank (as
    torch.distributed.broadcast takes it), also when `group` is a subgroup.  Returns the number of collectives."""
    calls = 0
    by_dtype: Dict[torch.dtype, List[str]] = {}
    for k in sorted(W):
        by_dtype.setdefault(W[k].dtype, []).append(k)
    for dt, names in by_dtype.items():
        i = 0
        while i < len(names):
            j, nbytes = i, 0
            while j < len(names) and (j == i or nbytes + W[names[j]].numel() * W[names[j]].element_size()
                                      <= bucket_bytes):
                nbytes += W[names[j]].numel() * W[names[j]].element_size()
                j += 1
            part = names[i:j]
            flat = torch.cat([W[k].reshape(-1) for k in part]) if len(part) > 1 else W[part[0]].reshape(-1).clone()
            dist.broadcast(flat, src, group=group)
            calls += 1
            if dist.get_rank() != src:  # global ranks on both sides (a subgroup's local numbering may differ)
                off = 0
                for k in part:
                    n = W[k].numel()
                    W[k].copy_(flat[off:off + n].view_as(W[k]))
                    off += n
            del flat
            i = j
    return calls


def gather_results(local: list, indices: List[int], total: int, dst: int = 0, group=None):
    """Host-side gather of per-rank results back into global order on `dst`, a GLOBAL rank as
    torch.distributed.gather_object takes it (None elsewhere)."""
    world = dist.get_world_size(group)
    payload = list(zip(indices, local))
    objs = [None] * world if dist.get_rank() == dst else None
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


def request_cost(input_ids, instruct_ids=None, frames=None, max_new_tokens=2048) -> List[int]:
    """LPT weight of each request: its expected decode frames (the caller's per-request estimate, else
    max_new_tokens) plus its prompt tokens -- decode dominates, a frame costs about as much as ~100 prompt
    tokens of prefill, so the prompt term only breaks ties."""
    n = len(input_ids)
    out = []
    for i in range(n):
        f = frames[i] if frames is not None else max_new_tokens
        p = int(torch.as_tensor(input_ids[i]).numel())
        if instruct_ids is not None and instruct_ids[i] is not None:
            p += int(torch.as_tensor(instruct_ids[i]).numel())
        out.append(100 * int(f) + p)
    return out


def dp_generate(model, input_ids, languages, speakers=None, instruct_ids=None, frames: Optional[Sequence[int]] = None,
                slots: int = 8, group=None, gather: bool = True, decode: bool = False, **gen):
    """Serve a request list data-parallel over the ranks of `group` (or alone when torch.distributed is not
    initialised): every rank takes its longest-first share of the requests (request_cost), decodes it through
    `slots` continuously refilled batch rows (TalkerEngine.serve via TTSModel.generate(max_batch=)), optionally
    decodes its PCM, and rank 0 gathers everything back into request order.

    model: a qwen_tts.model.TTSModel on this rank's GPU.  frames: optional per-request frame caps (known lengths /
    estimates); request i then stops after min(frames[i], max_new_tokens - 1) frames or at its EOS.  Each request
    draws Philox stream i (its global index), so sampled results do not depend on the rank count.
    Returns (codes list [F_i, 16], wavs list or None) on the group's rank 0 (every rank when gather=False returns its own
    share as {index: (codes, wav)}), None on other ranks."""
    world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
    rank = dist.get_rank(group) if world > 1 else 0
    n = len(input_ids)
    cost = request_cost(input_ids, instruct_ids, frames, gen.get("max_new_tokens", 2048))
    mine = shard_longest_first(cost, world)[rank]
    local = {}
    if mine:
        sub = lambda xs: None if xs is None else [xs[i] for i in mine]  # noqa: E731
        if frames is not None:
            gen = dict(gen, frame_caps=sub(frames))
        codes, _ = model.generate(input_ids=sub(input_ids), languages=sub(languages), speakers=sub(speakers),
                                  instruct_ids=sub(instruct_ids), max_batch=max(1, min(slots, len(mine))),
                                  philox_ids=mine, **gen)
        wavs = [None] * len(mine)
        if decode:
            wavs, _ = model.speech_tokenizer.decode([{"audio_codes": c} for c in codes])
            wavs = [w.cpu() if isinstance(w, torch.Tensor) else w for w in wavs]
        for j, i in enumerate(mine):
            local[i] = (codes[j], wavs[j])
    if not gather:
        return local
    if world == 1:
        res = [local[i] for i in range(n)]
    else:
        # rank 0 of `group`, as a global rank (the collective's dst); the shards above are by group rank
        dst = dist.get_global_rank(group, 0) if group is not None else 0
        res = gather_results([local[i] for i in mine], mine, n, dst=dst, group=group)
        if res is None:
            return None
    return [c for c, _ in res], ([w for _, w in res] if decode else None)
