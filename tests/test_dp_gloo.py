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
