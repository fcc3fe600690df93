"""World-size-2 gloo (CPU) coverage of the data-parallel path: sharding, weight broadcast, gather, timing."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from qwen_tts.dp import broadcast_weights, gather_results, reduce_timing, shard_longest_first


def test_shard_longest_first_balances():
    lens = [300, 40, 250, 64, 64, 120, 200, 90]
    sh = shard_longest_first(lens, 4)
    assert sorted(i for s in sh for i in s) == list(range(len(lens)))
    loads = [sum(lens[i] for i in s) for s in sh]
    assert max(loads) - min(loads) <= max(lens)
    assert shard_longest_first([5], 3) == [[0], [], []]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = torch.Generator().manual_seed(7)
    ref = {"a.weight": torch.randn(4, 3, generator=g), "b.bias": torch.randn(5, generator=g)}
    W = {k: (v.clone() if rank == 0 else torch.zeros_like(v)) for k, v in ref.items()}
    broadcast_weights(W)
    ok_w = all(torch.equal(W[k], ref[k]) for k in ref)
    lens = [30, 10, 25, 7, 12]
    mine = shard_longest_first(lens, world)[rank]
    res = gather_results([f"utt{i}@{rank}" for i in mine], mine, len(lens))
    dt, audio = reduce_timing(1.0 + rank, 10.0)
    if rank == 0:
        q.put((ok_w, res, dt, audio))
    dist.destroy_process_group()


def test_world2_gloo_broadcast_gather_timing():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    ok_w, res, dt, audio = q.get(timeout=120)
    for p in ps:
        p.join(timeout=60)
    assert ok_w
    assert [r.split("@")[0] for r in res] == [f"utt{i}" for i in range(5)]
    assert dt == 2.0 and audio == 20.0


class _StubModel:
    """Stands in for TTSModel on CPU: 'codes' encode the request's global id, so the gather order is checkable."""

    def __init__(self):
        self.calls = []

    def generate(self, input_ids, languages, speakers, instruct_ids, max_batch, philox_ids, frame_caps=None, **gen):
        self.calls.append(dict(n=len(input_ids), max_batch=max_batch, philox_ids=list(philox_ids), caps=frame_caps))
        codes = [torch.full((int(frame_caps[j]) if frame_caps else 3, 16), int(philox_ids[j])) for j in range(len(input_ids))]
        return codes, None


def _dp_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from qwen_tts.dp import dp_generate
    ids = [torch.zeros(1, n) for n in (5, 9, 3, 7, 11, 4, 6)]
    frames = [10, 40, 5, 30, 20, 8, 12]
    m = _StubModel()
    out = dp_generate(m, ids, ["english"] * 7, None, None, frames=frames, slots=2, max_new_tokens=64)
    # coalesced broadcast: mixed dtypes, a bucket limit that splits the fp32 tensors
    g = torch.Generator().manual_seed(3)
    ref = {"a": torch.randn(100, generator=g), "b": torch.randn(7, 3, generator=g), "c": torch.randn(50, generator=g),
           "d": torch.arange(6, dtype=torch.int64), "e": torch.randn(4, generator=g).to(torch.bfloat16)}
    W = {k: (v.clone() if rank == 0 else torch.zeros_like(v)) for k, v in ref.items()}
    calls = broadcast_weights(W, bucket_bytes=500)
    ok = all(torch.equal(W[k], ref[k]) for k in ref)
    q.put((rank, out, m.calls, ok, calls))
    dist.destroy_process_group()


def test_world2_dp_generate_shards_and_gathers():
    """dp_generate over 2 gloo ranks: each rank decodes its longest-first share with global Philox ids and frame caps,
    rank 0 gets every request back in order; the weight broadcast is coalesced per dtype into bounded buckets."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_dp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = dict((r[0], r[1:]) for r in (q.get(timeout=120), q.get(timeout=120)))
    for p in ps:
        p.join(timeout=60)
    out, calls0, ok, ncalls = got[0]
    assert got[1][0] is None and ok and got[1][2]
    codes, wavs = out
    frames = [10, 40, 5, 30, 20, 8, 12]
    assert wavs is None and len(codes) == 7
    for i, c in enumerate(codes):
        assert c.shape[0] == frames[i] and int(c[0, 0]) == i
    ids_all = sorted(calls0[0]["philox_ids"] + got[1][1][0]["philox_ids"])
    assert ids_all == list(range(7))
    loads = [sum(100 * frames[i] for i in c[0]["philox_ids"]) for c in (calls0, got[1][1])]
    assert abs(loads[0] - loads[1]) <= 100 * max(frames)
    assert ncalls == 4  # fp32 a+b (<= 500 B), fp32 c, int64 d, bf16 e


def _subgroup_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from qwen_tts.dp import dp_generate
    grp = dist.new_group([1, 2])  # collective on every rank; group-local ranks 0, 1 = global ranks 1, 2
    res = None
    if rank in (1, 2):
        ref = {"w": torch.arange(6, dtype=torch.float32) + 10.0}
        # global src 1 is group-local rank 0: rank 2 (local 1) must receive, rank 1 keeps its copy
        W = {"w": ref["w"].clone() if rank == 1 else torch.zeros(6)}
        broadcast_weights(W, src=1, group=grp)
        ids = [torch.zeros(1, n) for n in (5, 9, 3, 7)]
        out = dp_generate(_StubModel(), ids, ["english"] * 4, None, None, frames=[4, 9, 2, 6], slots=2,
                          max_new_tokens=64, group=grp)
        res = (torch.equal(W["w"], ref["w"]), None if out is None else [int(c[0, 0]) for c in out[0]])
    q.put((rank, res))
    dist.barrier()
    dist.destroy_process_group()


def test_world3_subgroup_uses_global_ranks():
    """A subgroup whose local numbering differs from the global one ([1, 2]): the weight broadcast from global rank 1
    reaches global rank 2, and dp_generate gathers to the group's first rank (global 1) in request order."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_subgroup_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(3))
    for p in ps:
        p.join(timeout=60)
    assert got[0] is None
    assert got[1] == (True, [0, 1, 2, 3])
    assert got[2] == (True, None)
