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
