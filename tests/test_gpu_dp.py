"""Data-parallel serving on the GPU path: per-utterance results of qwen_tts.dp.dp_generate over
2 ranks equal the 1-rank run.  Both ranks are spawned processes on cuda:0 (one GPU box) talking gloo for the host-side
gather -- the same code path the node runs with one rank per GPU over RCCL.  Sampling is on (each request draws the
Philox stream of its global index), with per-request frame caps, fp32 parity mode."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

N_REQ = 6
FRAMES = [9, 14, 5, 11, 7, 12]
GEN = dict(max_new_tokens=16, do_sample=True, subtalker_dosample=True, top_k=50, top_p=1.0, temperature=0.9,
           subtalker_top_k=50, subtalker_top_p=1.0, subtalker_temperature=0.9, repetition_penalty=1.05, seed=11,
           ignore_eos=True)


def _requests(cfg):
    from cases import text_ids
    ids = [text_ids(4 + 3 * i, 900 + i) for i in range(N_REQ)]
    spk = ["vivian", "ryan", "eric", "serena", "dylan", "aiden"][:N_REQ]
    return ids, ["english", "chinese", "auto", "english", "chinese", "english"][:N_REQ], spk


def _model():
    from oracle import load_preset, synth_state_dict, talker_param_specs
    from qwen_tts.model import TTSModel
    cfg, _ = load_preset("tiny-customvoice")
    W = {k: torch.from_numpy(v) for k, v in synth_state_dict(talker_param_specs(cfg)).items()}
    return cfg, TTSModel(cfg, W, dtype="fp32", device="cuda:0")


def _rank_main(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from qwen_tts.dp import dp_generate
        torch.cuda.set_device(0)
        cfg, m = _model()
        ids, langs, spk = _requests(cfg)
        out = dp_generate(m, ids, langs, spk, None, frames=FRAMES, slots=2, **GEN)
        if rank == 0:
            q.put(("ok", [c.numpy() for c in out[0]]))
        dist.destroy_process_group()
    except Exception as e:  # report instead of hanging the parent
        q.put(("err", repr(e)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_dp_two_ranks_equal_one_rank():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from qwen_tts.dp import dp_generate
    cfg, m = _model()
    ids, langs, spk = _requests(cfg)
    ref, _ = dp_generate(m, ids, langs, spk, None, frames=FRAMES, slots=2, **GEN)
    assert [c.shape[0] for c in ref] == FRAMES
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank_main, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    try:
        status, got = q.get(timeout=240)
    finally:
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert status == "ok", got
    assert len(got) == N_REQ
    for i, (a, b) in enumerate(zip(got, ref)):
        np.testing.assert_array_equal(a, b.numpy(), err_msg=f"request {i}")
