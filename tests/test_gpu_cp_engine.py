"""qt_cp_step (one persistent launch per code-predictor decode step: 5 layers + final norm + lm_head) against the
launch chain it replaces (qt_gemm q/k/v, the head-split qt_decode_attn_oproj, gate/up + SwiGLU, down, lm_head GEMV) on
the same inputs, at the code predictor's real dims (hidden 1024, 16 / 8 heads x 128, intermediate 3072, 5 layers,
2048 codes), bf16.  Both compute in bf16 MFMA with fp32 accumulation in different summation orders, so logits and the
appended K/V are compared within bf16 tolerance; the engine itself is deterministic (repeat launches give the same
bits), advances its launch counter across launches on one workspace (changing row counts and cache positions) and
never sets its hand-off error flag."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def _cp_stack(dev, seed=0):
    from oracle import load_preset
    from qwen_tts.talker import _Stack
    cfg, _ = load_preset("1.7b-customvoice")
    lc = cfg["talker_config"]["code_predictor_config"]
    g = torch.Generator().manual_seed(seed)
    H, I, D = lc["hidden_size"], lc["intermediate_size"], lc["head_dim"]
    nq, nkv = lc["num_attention_heads"], lc["num_key_value_heads"]
    W = {}
    r = lambda *s: (0.03 * torch.randn(*s, generator=g))  # noqa: E731
    n = lambda *s: (1 + 0.1 * torch.randn(*s, generator=g))  # noqa: E731
    for i in range(lc["num_hidden_layers"]):
        p = f"cp.layers.{i}"
        W[f"{p}.self_attn.q_proj.weight"] = r(nq * D, H)
        W[f"{p}.self_attn.k_proj.weight"] = r(nkv * D, H)
        W[f"{p}.self_attn.v_proj.weight"] = r(nkv * D, H)
        W[f"{p}.self_attn.o_proj.weight"] = r(H, nq * D)
        W[f"{p}.mlp.gate_proj.weight"] = r(I, H)
        W[f"{p}.mlp.up_proj.weight"] = r(I, H)
        W[f"{p}.mlp.down_proj.weight"] = r(H, I)
        W[f"{p}.input_layernorm.weight"] = n(H)
        W[f"{p}.post_attention_layernorm.weight"] = n(H)
        W[f"{p}.self_attn.q_norm.weight"] = n(D)
        W[f"{p}.self_attn.k_norm.weight"] = n(D)
    W["cp.norm.weight"] = n(H)
    st = _Stack(W, "cp", lc, torch.bfloat16, dev, 32)
    from qwen_tts import kernels as Kn
    lm = Kn.tile_linear((0.03 * torch.randn(lc["vocab_size"], H, generator=g)).to(dev), torch.bfloat16, gamma=st.norm)
    return st, lm, g


def _inputs(st, R, Lmax, g, dev):
    from qwen_tts import kernels as Kn
    x = torch.randn(R, st.H, generator=g).to(dev)
    x16 = x.to(torch.bfloat16)
    qkv0 = torch.empty(R, st.qkv_w, device=dev)
    Kn.gemm(x16, st.layers[0].qkv, qkv0, R, st.H, st.qkv_w, rms=True, eps=st.eps)
    kc = [torch.randn(R, st.Hkv, Lmax, st.D, generator=g).to(dev, torch.bfloat16) for _ in st.layers]
    vc = [torch.randn(R, st.Hkv, Lmax, st.D, generator=g).to(dev, torch.bfloat16) for _ in st.layers]
    return x, x16, qkv0, kc, vc


def _chain(st, lm, x, x16, qkv0, kc, vc, R, Lmax, pos, dev):
    """The launch chain of TalkerEngine._cp_lane for one decode step (qkv0 = layer 0's q/k/v rows)."""
    from qwen_tts import kernels as Kn
    from qwen_tts.talker import _scratch
    sc = _scratch(R, st, dev, attn_oproj=True)
    sc["qkv"][:R] = qkv0
    meta = {"const_pos": pos}
    st.forward(x, R, meta, (kc, vc), sc, Lmax, Lmax, decode=True, x16=x16, qkv0=True)
    logits = torch.empty(R, lm.N, device=dev)
    Kn.gemm(x16, lm, logits, R, st.H, lm.N, rms=True, eps=st.eps)
    return logits


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm())


@pytest.mark.parametrize("R,pos", [(8, 2), (8, 15), (5, 9), (1, 4)])
def test_cp_step_matches_launch_chain(R, pos):
    from qwen_tts import kernels as Kn
    dev = _dev()
    st, lm, g = _cp_stack(dev)
    if not Kn.cp_step_supported(st.H, st.I, st.Hq, st.Hkv, st.D, st.n_layers, lm.N):
        pytest.skip("qt_cp_step not supported on this device")
    Lmax = 18
    x, x16, qkv0, kc, vc = _inputs(st, R, Lmax, g, dev)
    kc1, vc1 = [k.clone() for k in kc], [v.clone() for v in vc]
    ref = _chain(st, lm, x.clone(), x16.clone(), qkv0, kc1, vc1, R, Lmax, pos, dev)
    ws = torch.zeros(Kn.cp_step_ws_bytes(), dtype=torch.uint8, device=dev)
    outs = []
    for _ in range(3):
        kc2, vc2 = [k.clone() for k in kc], [v.clone() for v in vc]
        logits = torch.full((R, lm.N), float("nan"), device=dev)
        Kn.cp_step(st.layers, lm, x, qkv0, R, kc2, vc2, Lmax, pos, st.cos, st.sin, st.eps, logits, ws)
        torch.cuda.synchronize()
        outs.append((logits, kc2, vc2))
    assert int(ws[:4].view(torch.int32).item()) == 0, "hand-off poll gave up"
    for o in outs[1:]:  # deterministic over launches (the tags advance)
        assert torch.equal(o[0], outs[0][0])
    logits, kc2, vc2 = outs[0]
    e = _rel(logits, ref)
    print(f"\n  R={R} pos={pos}: logits rel-L2 {e:.2e}, max|d| {float((logits - ref).abs().max()):.3g} "
          f"(|ref| max {float(ref.abs().max()):.3g}); argmax agree {(logits.argmax(-1) == ref.argmax(-1)).float().mean():.2f}")
    assert torch.isfinite(logits).all()
    # measured 5.7e-3 - 6.5e-3 (the engine's attention is fp32, the fused chain's attn_oproj_hs_k rounds q and the
    # softmax weights to bf16; tests/test_gpu_engine_stages.py pins each against fp64)
    assert e < 1e-2
    for li in range(st.n_layers):
        # layer 0's new key / value come from the same q/k/v rows: identical; later layers within bf16 rounding
        if li == 0:
            assert torch.equal(kc2[li], kc1[li]) and torch.equal(vc2[li], vc1[li])
        else:
            ek, ev = _rel(kc2[li][:, :, pos], kc1[li][:, :, pos]), _rel(vc2[li][:, :, pos], vc1[li][:, :, pos])
            print(f"  layer {li}: new key rel {ek:.2e}, value rel {ev:.2e}")
            assert ek < 1e-2 and ev < 1e-2
            assert torch.equal(kc2[li][:, :, :pos], kc1[li][:, :, :pos])  # nothing else written


def test_cp_step_launch_sequence_on_one_workspace():
    """14 consecutive decode steps (positions 2..15) and changing row counts on ONE workspace, each launch against the
    launch chain on the same inputs."""
    from qwen_tts import kernels as Kn
    dev = _dev()
    st, lm, g = _cp_stack(dev, seed=3)
    if not Kn.cp_step_supported(st.H, st.I, st.Hq, st.Hkv, st.D, st.n_layers, lm.N):
        pytest.skip("qt_cp_step not supported on this device")
    Lmax = 18
    ws = torch.zeros(Kn.cp_step_ws_bytes(), dtype=torch.uint8, device=dev)
    for i, (R, pos) in enumerate([(8, p) for p in range(2, 16)] + [(3, 7), (8, 3), (2, 12)]):
        x, x16, qkv0, kc, vc = _inputs(st, R, Lmax, g, dev)
        ref = _chain(st, lm, x.clone(), x16.clone(), qkv0, [k.clone() for k in kc], [v.clone() for v in vc], R, Lmax,
                     pos, dev)
        logits = torch.full((R, lm.N), float("nan"), device=dev)
        Kn.cp_step(st.layers, lm, x, qkv0, R, kc, vc, Lmax, pos, st.cos, st.sin, st.eps, logits, ws)
        assert _rel(logits, ref) < 1e-2, (i, R, pos, _rel(logits, ref))
    epoch = int(ws[4:8].view(torch.int32).item())
    assert epoch == 17
    assert int(ws[:4].view(torch.int32).item()) == 0


def _prefill_chain(st, lm, x, R, kc, vc, Lmax, dev):
    """The launch chain of TalkerEngine._cp_lane's 2-token prefill: rows (2b, 2b + 1) at positions 0, 1 through every
    layer (attn_small_prefill_k), then lm_head[0] on the odd rows."""
    from qwen_tts import kernels as Kn
    from qwen_tts.talker import _scratch
    i32 = lambda t: t.to(torch.int32).to(dev)  # noqa: E731
    p2 = i32(torch.arange(2 * R) % 2)
    meta = {"rope_pos": p2, "kv_pos": p2.clone(), "row_len": p2 + 1, "row_start": i32(torch.zeros(2 * R)),
            "row_batch": i32(torch.arange(2 * R) // 2), "small_T": 2}
    x16 = x.to(torch.bfloat16)
    st.forward(x, 2 * R, meta, (kc, vc), _scratch(2 * R, st, dev, attn_oproj=True), Lmax, Lmax, x16=x16)
    logits = torch.empty(R, lm.N, device=dev)
    Kn.gemm(x16.view(-1)[st.H:], lm, logits, R, 2 * st.H, lm.N, rms=True, eps=st.eps)
    return logits


@pytest.mark.parametrize("R", [8, 5, 1])
def test_cp_prefill_matches_launch_chain(R):
    """qt_cp_prefill (16 token rows through the step engine) against the prefill launch chain: logits of position 1
    and the keys / values appended at positions 0, 1 within bf16 tolerance; deterministic; on a workspace shared with
    decode steps."""
    from qwen_tts import kernels as Kn
    dev = _dev()
    st, lm, g = _cp_stack(dev, seed=5)
    if not Kn.cp_step_supported(st.H, st.I, st.Hq, st.Hkv, st.D, st.n_layers, lm.N):
        pytest.skip("qt_cp_step not supported on this device")
    Lmax = 18
    x = torch.randn(2 * R, st.H, generator=g).to(dev)
    kc = [torch.randn(R, st.Hkv, Lmax, st.D, generator=g).to(dev, torch.bfloat16) for _ in st.layers]
    vc = [torch.randn(R, st.Hkv, Lmax, st.D, generator=g).to(dev, torch.bfloat16) for _ in st.layers]
    kc1, vc1 = [k.clone() for k in kc], [v.clone() for v in vc]
    ref = _prefill_chain(st, lm, x.clone(), R, kc1, vc1, Lmax, dev)
    ws = torch.zeros(Kn.cp_step_ws_bytes(), dtype=torch.uint8, device=dev)
    outs = []
    for i in range(3):
        if i == 1:  # a decode step in between on the same workspace
            xd, x16d, qkv0, kcd, vcd = _inputs(st, R, Lmax, g, dev)
            Kn.cp_step(st.layers, lm, xd, qkv0, R, kcd, vcd, Lmax, 2, st.cos, st.sin, st.eps,
                       torch.empty(R, lm.N, device=dev), ws)
        kc2, vc2 = [k.clone() for k in kc], [v.clone() for v in vc]
        logits = torch.full((R, lm.N), float("nan"), device=dev)
        Kn.cp_prefill(st.layers, lm, x, R, kc2, vc2, Lmax, st.cos, st.sin, st.eps, logits, ws)
        torch.cuda.synchronize()
        outs.append((logits, kc2, vc2))
    assert int(ws[:4].view(torch.int32).item()) == 0, "hand-off poll gave up"
    for o in outs[1:]:
        assert torch.equal(o[0], outs[0][0])
    logits, kc2, vc2 = outs[0]
    e = _rel(logits, ref)
    print(f"\n  prefill R={R}: logits rel-L2 {e:.2e}; argmax agree {(logits.argmax(-1) == ref.argmax(-1)).float().mean():.2f}")
    assert torch.isfinite(logits).all()
    assert e < 5e-3  # measured 2.6e-3 - 3.4e-3
    for li in range(st.n_layers):
        for t in range(2):
            ek, ev = _rel(kc2[li][:, :, t], kc1[li][:, :, t]), _rel(vc2[li][:, :, t], vc1[li][:, :, t])
            print(f"  layer {li} position {t}: key rel {ek:.2e}, value rel {ev:.2e}")
            assert ek < 5e-3 and ev < 5e-3, (li, t, ek, ev)
        assert torch.equal(kc2[li][:, :, 2:], kc1[li][:, :, 2:])  # nothing else written
        assert torch.equal(vc2[li][:, :, 2:], vc1[li][:, :, 2:])
    assert int(ws[4:8].view(torch.int32).item()) == 4  # 3 prefills + 1 decode step advanced the launch counter


@pytest.mark.parametrize("R,do_sample,force,top_k,top_p", [(8, True, False, 50, 1.0), (5, True, True, 50, 1.0),
                                                            (3, False, False, 50, 1.0), (8, True, False, 200, 0.8),
                                                            (4, True, False, 0, 1.0)])
def test_cp_step_sampled_equals_sample_then_step(R, do_sample, force, top_k, top_p):
    """qt_cp_step_sampled (the previous step's qt_sample body run inside the engine launch, the chosen rows handed over
    in-launch) against qt_sample followed by qt_cp_step on the same logits / tables / counters: the same tokens, codes
    and teacher-forcing picks, and bit-identical logits and appended K/V (the engine sees the same input rows).  The
    sampler paths: top-k 50 (histogram / per-wave candidates + Gumbel-max), top-k 200 with top-p 0.8 (the sorted
    nucleus cut in the engine's LDS), no top-k (inverse CDF over the whole vocabulary), greedy."""
    from qwen_tts import kernels as Kn
    dev = _dev()
    st, lm, g = _cp_stack(dev, seed=7)
    if not Kn.cp_step_supported(st.H, st.I, st.Hq, st.Hkv, st.D, st.n_layers, lm.N):
        pytest.skip("qt_cp_step not supported on this device")
    Lmax, V, pos, G = 18, lm.N, 6, 16
    prev_logits = (torch.randn(R, V, generator=g) * 3).to(dev)
    tab_x = torch.randn(V, st.H, generator=g).to(dev)
    tab_q = torch.randn(V, st.qkv_w, generator=g).to(dev)
    kc = [torch.randn(R, st.Hkv, Lmax, st.D, generator=g).to(dev, torch.bfloat16) for _ in st.layers]
    vc = [torch.randn(R, st.Hkv, Lmax, st.D, generator=g).to(dev, torch.bfloat16) for _ in st.layers]
    step = torch.tensor([3, 1, 4, 1, 5, 9, 2, 6][:R], dtype=torch.int32, device=dev)
    prow = torch.arange(10, 10 + R, dtype=torch.int32, device=dev)
    seed = torch.tensor([1234567], dtype=torch.int64, device=dev)
    frc = torch.randint(0, V, (R, 12 * G), generator=g, dtype=torch.int32).to(dev) if force else None

    def run(fused):
        codes = torch.full((R, 12 * G), -1, dtype=torch.int32, device=dev)
        pick = torch.full((R, 12 * G), -1, dtype=torch.int32, device=dev) if force else None
        tok = torch.full((R,), -1, dtype=torch.int32, device=dev)
        x = torch.zeros(R, st.H, device=dev)
        q0 = torch.zeros(R, st.qkv_w, device=dev)
        k2, v2 = [k.clone() for k in kc], [v.clone() for v in vc]
        logits = torch.full((R, V), float("nan"), device=dev)
        ws = torch.zeros(Kn.cp_step_ws_bytes(), dtype=torch.uint8, device=dev)
        sa = Kn.sample(prev_logits, R, V, V, tok, do_sample=do_sample, top_k=top_k, top_p=top_p, temperature=0.9,
                       seed_ptr=seed, step=step, substep=pos, codes=codes, codes_ld=12 * G, codes_w=G,
                       codes_col=pos - 1, codes_step_off=0, ctr_stride=1, philox_row=prow, emb=(tab_x, x, st.H),
                       emb2=(tab_q, q0, st.qkv_w), force=frc, pick=pick, launch=not fused)
        Kn.cp_step(st.layers, lm, x, q0, R, k2, v2, Lmax, pos, st.cos, st.sin, st.eps, logits, ws,
                   sample=sa if fused else None)
        torch.cuda.synchronize()
        assert int(ws[:4].view(torch.int32).item()) == 0, "hand-off poll gave up"
        return tok, codes, pick, logits, k2, v2

    ref, fus = run(False), run(True)
    print(f"\n  R={R} sample={do_sample} force={force} top_k={top_k} top_p={top_p}: tokens {ref[0].tolist()} / "
          f"{fus[0].tolist()}")
    assert torch.equal(ref[0], fus[0]) and torch.equal(ref[1], fus[1])
    if force:
        assert torch.equal(ref[2], fus[2])
    assert torch.equal(ref[3], fus[3])
    for a, b in zip(ref[4] + ref[5], fus[4] + fus[5]):
        assert torch.equal(a, b)
