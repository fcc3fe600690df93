"""The head-split code-predictor attention + o_proj (attn_oproj_hs_k) hands row partials between blocks of one launch:
residency of its grid, behaviour beside a concurrent kernel on another stream, and the host side of its sticky
give-up flag (checked and cleared per request / per streamed chunk, so a pooled session serves its next request)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def test_head_split_grid_is_resident():
    """Every block of the code predictor's head-split grid ((1024 / 32) x 8 = 256) fits on the device at once (the
    dispatcher checks the same occupancy figure before choosing that form)."""
    from qwen_tts import _hip
    _dev()
    n = _hip.lib().qt_attn_oproj_resident_blocks()
    print(f"\n  head-split kernel: {n} resident blocks on this device")
    assert n >= 256


def test_head_split_beside_concurrent_kernel():
    """Head-split launches issued while a long GEMM stream runs on a second stream (its blocks compete for the CUs
    while the consumer blocks poll): every output equals the idle-GPU result bit for bit and the flag stays clear."""
    from qwen_tts import kernels as Kn
    dev = _dev()
    D, hq, hkv, N, B, Lmax, pos = 128, 16, 8, 1024, 8, 18, 9
    g = torch.Generator().manual_seed(31)
    qn, kn = (1 + 0.1 * torch.randn(D, generator=g)).to(dev), (1 + 0.1 * torch.randn(D, generator=g)).to(dev)
    wo = Kn.tile_linear((torch.randn(N, hq * D, generator=g) * 0.05).to(dev), torch.bfloat16)
    cos, sin = Kn.rope_tables(D, 1e6, Lmax + 8, dev)
    qkv = torch.randn(B, (hq + 2 * hkv) * D, generator=g).to(dev)
    kc = torch.randn(B, hkv, Lmax, D, generator=g).to(dev, torch.bfloat16)
    vc = torch.randn(B, hkv, Lmax, D, generator=g).to(dev, torch.bfloat16)
    x0 = torch.randn(B, N, generator=g).to(dev)
    ws = torch.zeros(Kn.attn_oproj_ws_bytes(N, hkv), dtype=torch.uint8, device=dev)

    def one():
        x = x0.clone()
        Kn.decode_attn_oproj(qkv, B, hq, hkv, D, qn, kn, 1e-6, cos, sin, kc.clone(), vc.clone(), Lmax, wo, x,
                             const_pos=pos, ws=ws)
        return x
    ref = one()
    torch.cuda.synchronize()
    # the competing work: a prefill-sized GEMM chain (~ms) on a side stream
    M, K_, Nn = 4096, 2048, 6144
    A = torch.randn(M, K_, device=dev).to(torch.bfloat16)
    Wb = Kn.tile_linear(torch.randn(Nn, K_, device=dev) * 0.02, torch.bfloat16)
    C = torch.empty(M, Nn, dtype=torch.bfloat16, device=dev)
    side = torch.cuda.Stream(device=dev)
    outs = []
    with torch.cuda.stream(side):
        for _ in range(20):
            Kn.gemm(A, Wb, C, M, K_, Nn)
    for _ in range(64):
        outs.append(one())
    torch.cuda.synchronize()
    for x in outs:
        assert torch.equal(x, ref)
    assert int(ws[:4].view(torch.int32).item()) == 0


def _model_06b():
    from oracle import load_preset, synth_state_dict, talker_param_specs
    from qwen_tts.model import TTSModel
    cfg, _ = load_preset("0.6b-customvoice")
    W = {k: torch.from_numpy(v) for k, v in synth_state_dict(talker_param_specs(cfg), threads=16).items()}
    return TTSModel(cfg, W, dtype="bf16")


def test_handoff_flag_raises_then_session_is_reused():
    """A set flag fails the request that ran with it (generate at its end, stream() before the chunk whose frames it
    covers is handed out) and is cleared, so the pooled session's next request decodes normally (same codes)."""
    from qwen_tts.talker import HANDOFF_ERROR
    _dev()
    m = _model_06b()
    ids = [torch.tensor([[151644, 77091, 198] + list(range(1000, 1040)) + [151645, 198, 151644, 77091, 198]])]
    kw = dict(input_ids=ids, languages=["english"], speakers=["vivian"], non_streaming_mode=True, do_sample=False,
              subtalker_dosample=False, max_new_tokens=12, ignore_eos=True)
    base, _ = m.generate(**kw)
    ss = [s for s in m.engine.all_sessions() if s.cp.sc.get("ao_ws") is not None]
    assert ss, "the bf16 0.6B code predictor should take the head-split form"
    for s in ss:
        s.cp.sc["ao_ws"][:4].view(torch.int32).fill_(1)
    with pytest.raises(RuntimeError, match="hand-off timed out"):
        m.generate(**kw)
    assert all(int(s.cp.sc["ao_ws"][:4].view(torch.int32).item()) == 0 for s in ss)
    again, _ = m.generate(**kw)
    assert all(torch.equal(a, b) for a, b in zip(base, again))
    # the code-predictor step engine's own flag (qt_cp_step workspace)
    ce = [s for s in ss if s.cp.ce_ws is not None]
    if ce:
        for s in ce:
            s.cp.ce_ws[:4].view(torch.int32).fill_(1)
        with pytest.raises(RuntimeError, match="hand-off timed out"):
            m.generate(**kw)
        assert all(int(s.cp.ce_ws[:4].view(torch.int32).item()) == 0 for s in ce)
        again, _ = m.generate(**kw)
        assert all(torch.equal(a, b) for a, b in zip(base, again))
    # a streamed decode (decode_iter, as stream() drives it): the flag set while frames decode is reported at the next
    # chunk boundary, before that chunk's frames are handed out
    from qwen_tts.talker import GenParams
    emb, mask, trail, pad = m.build_prompts(ids, ["english"], ["vivian"], None, True)
    gp = GenParams(max_new_tokens=12, do_sample=False, subtalker_dosample=False, ignore_eos=True)
    chunks = 0
    with pytest.raises(RuntimeError, match="hand-off timed out"):
        for sessions, frames, final in m.engine.decode_iter(emb, mask, trail, pad, gp, every=2, first=1):
            chunks += 1
            for s in sessions:
                s.cp.sc["ao_ws"][:4].view(torch.int32).fill_(1)
    assert chunks >= 1
    assert "in-launch hand-off" in HANDOFF_ERROR
    again2, _ = m.generate(**kw)
    assert all(torch.equal(a, b) for a, b in zip(base, again2))


def test_engines_beside_concurrent_codec_kernels():
    """VERDICT r05 "do this" 3 / ADVICE r05: the persistent engines (qt_cp_step: 14 decode steps of a frame, qt_cp_prefill,
    qt_talker_tail: 28 layer tails) launched on the main stream while a long window of codec implicit-GEMM launches
    (igemm_k, fp32 activations x bf16 weights, as the voice-clone stream() decodes reference frames on a side stream,
    model.py _start_ref_decode) runs on a second stream: the engines' 256 workgroups become resident as the codec blocks
    drain, every output is bit-identical to the idle-GPU run, and no hand-off flag is set."""
    import sys
    import os
    sys.path.insert(0, os.path.dirname(__file__))
    from test_gpu_cp_engine import _cp_stack, _inputs
    from test_gpu_talker_tail import _layers, _inputs as _tt_inputs, H as TH, I as TI, HQ, D as TD, QKV
    from qwen_tts import kernels as Kn
    dev = _dev()
    st, lm, g = _cp_stack(dev, seed=13)
    if not (Kn.cp_step_supported(st.H, st.I, st.Hq, st.Hkv, st.D, st.n_layers, lm.N)
            and Kn.talker_tail_supported(TH, TI, HQ, TD, QKV)):
        pytest.skip("engines not supported on this device")
    R, Lmax = 8, 18
    x, x16, qkv0, kc, vc = _inputs(st, R, Lmax, g, dev)
    xp = torch.randn(2 * R, st.H, generator=g).to(dev)
    L, Ln = _layers(dev)
    att, xt = _tt_inputs(R, dev, seed=9)

    def run():
        ws_c = torch.zeros(Kn.cp_step_ws_bytes(), dtype=torch.uint8, device=dev)
        ws_t = torch.zeros(Kn.talker_tail_ws_bytes(), dtype=torch.uint8, device=dev)
        k2, v2 = [k.clone() for k in kc], [v.clone() for v in vc]
        outs = []
        lg = torch.empty(R, lm.N, device=dev)
        Kn.cp_prefill(st.layers, lm, xp, R, k2, v2, Lmax, st.cos, st.sin, st.eps, lg, ws_c)
        outs.append(lg)
        for pos in range(2, 16):
            lg = torch.empty(R, lm.N, device=dev)
            Kn.cp_step(st.layers, lm, x, qkv0, R, k2, v2, Lmax, pos, st.cos, st.sin, st.eps, lg, ws_c)
            outs.append(lg)
        xe = xt.clone()
        for i in range(28):
            q = torch.empty(R, QKV, device=dev)
            Kn.talker_tail(att, xe, R, L, Ln if i % 2 == 0 else None, q, 1e-6, ws_t)
            if i % 2 == 0:
                outs.append(q)
        outs += [xe] + k2 + v2
        return outs, ws_c, ws_t

    ref, _, _ = run()
    torch.cuda.synchronize()
    # the codec window: 1-D conv-sized implicit GEMMs (fp32 A, bf16 weights -> igemm_k), ~tens of ms on the side stream
    M, K_, N = 8192, 1536, 1536
    A = torch.randn(M, K_, device=dev)
    Wc = Kn.tile_linear(torch.randn(N, K_, device=dev) * 0.02, torch.bfloat16)
    C = torch.empty(M, N, device=dev)
    side = Kn.side_stream(dev)
    for trial in range(3):
        with torch.cuda.stream(side):
            for _ in range(40):
                Kn.gemm(A, Wc, C, M, K_, N)
        got, ws_c, ws_t = run()
        torch.cuda.synchronize()
        assert int(ws_c[:4].view(torch.int32).item()) == 0, "cp engine hand-off gave up beside the codec kernels"
        assert int(ws_t[:4].view(torch.int32).item()) == 0, "talker tail hand-off gave up beside the codec kernels"
        for a, b in zip(got, ref):
            assert torch.equal(a, b)


def test_concurrent_requests_on_two_streams():
    """Two requests decoding at once from two streams (their frames interleaved on the host, each on its own stream,
    as two serving threads would issue them): every frame's persistent engines run without the other request's engines
    beside them (TalkerEngine._fence_in / _fence_out), so both give the codes they give alone and no flag is set."""
    from qwen_tts.talker import GenParams
    _dev()
    m = _model_06b()
    mk = lambda lo, n: torch.tensor([[151644, 77091, 198] + list(range(lo, lo + n)) + [151645, 198, 151644, 77091, 198]])  # noqa: E731
    reqs = [([mk(1000, 40), mk(3000, 25)], ["english", "chinese"], ["vivian", "ryan"]),
            ([mk(5000, 33)], ["english"], ["serena"])]
    gp = GenParams(max_new_tokens=24, do_sample=False, subtalker_dosample=False, ignore_eos=True)
    alone = [m.generate(input_ids=ids, languages=lg, speakers=sp, non_streaming_mode=True, do_sample=False,
                        subtalker_dosample=False, max_new_tokens=24, ignore_eos=True)[0] for ids, lg, sp in reqs]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    its, outs = [], [None, None]
    for (ids, lg, sp), st in zip(reqs, streams):
        emb, mask, trail, pad = m.build_prompts(ids, lg, sp, None, True)
        its.append(m.engine.decode_iter(emb, mask, trail, pad, gp, every=1, first=1))
    live = [0, 1]
    while live:
        for i in list(live):
            with torch.cuda.stream(streams[i]):
                sessions, frames, final = next(its[i])
                if final:
                    outs[i] = m.engine.collect(sessions, frames)[0]
                    its[i].close()
                    live.remove(i)
    torch.cuda.synchronize()
    for a, b in zip(outs, alone):
        assert len(a) == len(b) and all(torch.equal(x, y) for x, y in zip(a, b))
