"""Stage-by-stage pin of the persistent engines against an fp64 PyTorch reference (VERDICT r05 "do this" 2).

qt_cp_step / qt_cp_prefill (csrc/cp_engine.hip) and qt_talker_tail (csrc/talker_tail.hip) record every stage's output
in a debug region past their workspace (qt_cp_step_dbg_bytes / qt_talker_tail_dbg_bytes).  The launch chain they
replace is run stage by stage on the same inputs, in its unfused form (qt_gemm GEMVs + qt_decode_attention /
qt_small_prefill_attention, as talker._Stack.forward issues them without the fused attention + o_proj, whose attention
rows are not observable).  For each stage of each layer the reference recomputes that stage in fp64 from the SAME
path's own input to it (its previous stage's recorded output) and the same bf16 weights (RMSNorm gammas folded and
rounded as kernels.tile_linear / tile_swiglu do), so the error measured is the stage's own, not inherited:

    q/k/v      rms(bf16(x)) @ W_qkv^T                                             (M:985, M:752-754)
    attention  q/k RMSNorm + RoPE + softmax(q k^T / sqrt(D)) v over the cache + the new key   (M:740-804, 764-765)
    x_attn     x + attention @ W_o^T  (the path's own bf16 attention rows)                   (M:804, 991)
    h          silu(rms(bf16(x_attn)) @ W_gate^T) * (rms(bf16(x_attn)) @ W_up^T)     (M:993-1001)
    x_mlp      x_attn + bf16(h) @ W_down^T                                           (M:1004)
    logits     rms(bf16(x_mlp of the last layer)) @ W_lm^T  (final norm folded)      (M:1142, 1299)

Errors are rel-L2 of the stage's increment (residual stages: relative to ref - x_in).  Asserted per stage and layer:
the engine's error <= 1.25 x the launch chain's error (+ 1e-6), and below 1e-2 (the attention and SwiGLU outputs are
stored in bf16: ~1e-3 - 2e-3 of rounding; the fp32 stages sit near 1e-7)."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

RATIO, FLOOR = 1.25, 1e-6


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def _bf(t):
    return t.to(torch.bfloat16).double()


def _rel(a, ref, base=None):
    d = ref.double() if base is None else ref.double() - base.double()
    return float((a.double() - ref.double()).norm() / d.norm())


def _rms_lin(x, w_eff, eps):
    a = _bf(x)
    rs = torch.rsqrt((a * a).mean(-1, keepdim=True) + eps)
    return (a @ w_eff.double().T) * rs


def _swiglu_ref(x, wg, wu, eps):
    a = _bf(x)
    rs = torch.rsqrt((a * a).mean(-1, keepdim=True) + eps)
    g, u = (a @ wg.double().T) * rs, (a @ wu.double().T) * rs
    return torch.nn.functional.silu(g) * u


def _qk_rope(t, w, c, s, eps):
    t = t * torch.rsqrt((t * t).mean(-1, keepdim=True) + eps) * w.double()
    h = t.shape[-1] // 2
    t1, t2 = t[..., :h], t[..., h:]
    return torch.cat([t1 * c - t2 * s, t2 * c + t1 * s], -1)


def _attn_decode_ref(qkv, kc, vc, pos, qn, kn, cos, sin, Hq, Hkv, D, eps):
    """One new token per row at cache position pos (cached keys [0, pos) + the new one, bf16 as the cache holds them)."""
    R = qkv.shape[0]
    q = qkv[:, :Hq * D].double().view(R, Hq, D)
    k = qkv[:, Hq * D:(Hq + Hkv) * D].double().view(R, Hkv, D)
    v = qkv[:, (Hq + Hkv) * D:].double().view(R, Hkv, D)
    c, s = cos[pos].double(), sin[pos].double()
    q, k = _qk_rope(q, qn, c, s, eps), _qk_rope(k, kn, c, s, eps)
    K = torch.cat([kc[:R, :, :pos].double(), _bf(k)[:, :, None]], 2).repeat_interleave(Hq // Hkv, 1)
    V = torch.cat([vc[:R, :, :pos].double(), _bf(v)[:, :, None]], 2).repeat_interleave(Hq // Hkv, 1)
    p = torch.softmax((q[:, :, None, :] * K).sum(-1) / math.sqrt(D), -1)
    return (p[..., None] * V).sum(2).reshape(R, Hq * D)


def _attn_prefill_ref(qkv, qn, kn, cos, sin, Hq, Hkv, D, eps):
    """Token rows (2b, 2b + 1) = positions 0, 1 of batch row b, causal over the two new keys (bf16-rounded)."""
    R2 = qkv.shape[0]
    q = qkv[:, :Hq * D].double().view(R2, Hq, D)
    k = qkv[:, Hq * D:(Hq + Hkv) * D].double().view(R2, Hkv, D)
    v = qkv[:, (Hq + Hkv) * D:].double().view(R2, Hkv, D)
    pos = torch.arange(R2, device=qkv.device) % 2
    c, s = cos[pos].double()[:, None], sin[pos].double()[:, None]
    q, k = _qk_rope(q, qn, c, s, eps), _bf(_qk_rope(k, kn, c, s, eps))
    v = _bf(v)
    out = torch.empty(R2, Hq, D, dtype=torch.float64, device=qkv.device)
    for r in range(R2):
        b0 = r - r % 2
        K = k[b0:r + 1].repeat_interleave(Hq // Hkv, 1)  # [t + 1, Hq, D]
        V = v[b0:r + 1].repeat_interleave(Hq // Hkv, 1)
        p = torch.softmax((q[r][None] * K).sum(-1) / math.sqrt(D), 0)  # [t + 1, Hq]
        out[r] = (p[..., None] * V).sum(0)
    return out.reshape(R2, Hq * D)


# ---------------------------------------------------------------------------------------------- code predictor
class _CP:
    """The code predictor at its real dims (hidden 1024, 16 / 8 heads x 128, intermediate 3072, 5 layers, 2048 codes):
    raw weights (for the reference) and the tiled _Stack the kernels read."""

    def __init__(self, dev, seed=0):
        from oracle import load_preset
        from qwen_tts import kernels as Kn
        from qwen_tts.talker import _Stack
        cfg, _ = load_preset("1.7b-customvoice")
        lc = cfg["talker_config"]["code_predictor_config"]
        g = torch.Generator().manual_seed(seed)
        H, I, D = lc["hidden_size"], lc["intermediate_size"], lc["head_dim"]
        nq, nkv = lc["num_attention_heads"], lc["num_key_value_heads"]
        r = lambda *s: (0.03 * torch.randn(*s, generator=g))  # noqa: E731
        n = lambda *s: (1 + 0.1 * torch.randn(*s, generator=g))  # noqa: E731
        W = {}
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
        self.st = st = _Stack(W, "cp", lc, torch.bfloat16, dev, 32)
        lm_raw = 0.03 * torch.randn(lc["vocab_size"], H, generator=g)
        self.lm = Kn.tile_linear(lm_raw.to(dev), torch.bfloat16, gamma=st.norm)
        self.g = g
        d = lambda t: t.to(dev)  # noqa: E731
        eff = lambda w, gam: (d(w).float() * d(gam).float()[None, :]).to(torch.bfloat16)  # noqa: E731
        self.ref = []
        for i in range(st.n_layers):
            p = f"cp.layers.{i}"
            wqkv = torch.cat([W[f"{p}.self_attn.{k}_proj.weight"] for k in "qkv"], 0)
            self.ref.append(dict(
                qkv=eff(wqkv, W[f"{p}.input_layernorm.weight"]), o=d(W[f"{p}.self_attn.o_proj.weight"]).to(torch.bfloat16),
                gate=eff(W[f"{p}.mlp.gate_proj.weight"], W[f"{p}.post_attention_layernorm.weight"]),
                up=eff(W[f"{p}.mlp.up_proj.weight"], W[f"{p}.post_attention_layernorm.weight"]),
                down=d(W[f"{p}.mlp.down_proj.weight"]).to(torch.bfloat16),
                qn=d(W[f"{p}.self_attn.q_norm.weight"]), kn=d(W[f"{p}.self_attn.k_norm.weight"])))
        self.lm_eff = eff(lm_raw, W["cp.norm.weight"])


def _cp_chain_staged(cp, x, x16, qkv0, kc, vc, R, Lmax, pos, dev):
    """The launch chain of one decode step in its unfused form (talker._Stack.forward with ATTN_OPROJ off: qt_gemm
    q/k/v, qt_decode_attention, o_proj + residual, gate/up + SwiGLU, down, lm_head), every stage's output recorded --
    the fused head-split attention + o_proj does not expose the attention rows; tests/test_gpu_cp_engine.py compares
    the engine with that fused chain end to end."""
    from qwen_tts import _hip, kernels as Kn
    from qwen_tts.talker import _scratch
    st = cp.st
    sc = _scratch(R, st, dev)
    rec = {"qkv": [], "att": [], "x_attn": [], "h": [], "x_mlp": []}
    i32 = lambda v: torch.full((R,), v, dtype=torch.int32, device=dev)  # noqa: E731
    pos_r, rb, zero = i32(pos), torch.arange(R, dtype=torch.int32, device=dev), i32(0)
    for li, L in enumerate(st.layers):
        if li == 0:
            sc["qkv"][:R] = qkv0
        else:
            Kn.gemm(x16, L.qkv, sc["qkv"], R, st.H, st.qkv_w, rms=True, eps=st.eps)
        rec["qkv"].append(sc["qkv"][:R].clone())
        Kn.decode_attention(sc["qkv"], R, st.Hq, st.Hkv, st.D, L.q_norm, L.k_norm, st.eps, st.cos, st.sin, pos_r, rb,
                            pos_r, zero, kc[li], vc[li], Lmax, sc["att"])
        rec["att"].append(sc["att"][:R].float())
        Kn.gemm(sc["att"], L.o, x, R, st.Hq * st.D, st.H, epi=_hip.EPI_ADD, out2=x16)
        rec["x_attn"].append(x.clone())
        Kn.gemm(x16, L.gu, sc["h"], R, st.H, st.I, rms=True, eps=st.eps, epi=_hip.EPI_SWIGLU)
        rec["h"].append(sc["h"][:R].float())
        Kn.gemm(sc["h"], L.down, x, R, st.I, st.H, epi=_hip.EPI_ADD, out2=x16)
        rec["x_mlp"].append(x.clone())
    logits = torch.empty(R, cp.lm.N, device=dev)
    Kn.gemm(x16, cp.lm, logits, R, st.H, cp.lm.N, rms=True, eps=st.eps)
    rec["logits"] = logits
    return rec


def _engine_rec(ws, nws, n_layers, rows):
    d = ws[nws:].view(torch.float32)[:6 * 5 * 16 * 4096].view(6, 5, 16, 4096)
    st = lambda k, w: [d[li, k, :rows, :w].clone() for li in range(n_layers)]  # noqa: E731
    return st


def _stage_errors(cp, rec, x_in, kc, vc, pos, R, prefill=False):
    """Per layer and stage: the stage's own error against fp64 recomputed from this path's input to it."""
    st, out = cp.st, []
    xin = x_in
    for li in range(st.n_layers):
        P = cp.ref[li]
        e = {}
        if li > 0 or prefill:
            e["qkv"] = _rel(rec["qkv"][li], _rms_lin(xin, P["qkv"], st.eps))
        if prefill:
            att = _attn_prefill_ref(rec["qkv"][li], P["qn"], P["kn"], st.cos, st.sin, st.Hq, st.Hkv, st.D, st.eps)
        else:
            att = _attn_decode_ref(rec["qkv"][li], kc[li], vc[li], pos, P["qn"], P["kn"], st.cos, st.sin, st.Hq, st.Hkv,
                                   st.D, st.eps)
        a_path = rec["att"][li][:, :st.Hq * st.D]  # (bf16 values)
        e["att"] = _rel(a_path, att)
        ref = xin.double() + a_path.double() @ P["o"].double().T  # o_proj + residual from the path's own attention rows
        e["x_attn"] = _rel(rec["x_attn"][li], ref, xin)
        xa = rec["x_attn"][li]
        e["h"] = _rel(rec["h"][li][:, :st.I], _swiglu_ref(xa, P["gate"], P["up"], st.eps))
        ref = xa.double() + _bf(rec["h"][li][:, :st.I]) @ P["down"].double().T
        e["x_mlp"] = _rel(rec["x_mlp"][li], ref, xa)
        xin = rec["x_mlp"][li]
        out.append(e)
    last = xin[1::2] if prefill else xin
    return out, _rel(rec["logits"], _rms_lin(last, cp.lm_eff, st.eps))


def _assert_ratio(eng, chain, tag, bound=1e-2):
    lines = []
    for li, (a, b) in enumerate(zip(eng[0], chain[0])):
        lines.append(f"  layer {li}: " + "  ".join(f"{k} {a[k]:.2e}/{b[k]:.2e}" if k in b else f"{k} {a[k]:.2e}"
                                                  for k in a))
    lines.append(f"  logits {eng[1]:.2e}/{chain[1]:.2e}")
    print(f"\n  {tag} (engine / chain error vs fp64, per stage)\n" + "\n".join(lines))
    for li, (a, b) in enumerate(zip(eng[0], chain[0])):
        for k in a:
            assert a[k] < bound, (tag, li, k, a[k])
            if k in b:
                assert a[k] <= RATIO * b[k] + FLOOR, (tag, li, k, a[k], b[k])
    assert eng[1] <= RATIO * chain[1] + FLOOR and eng[1] < bound, (tag, eng[1], chain[1])


@pytest.mark.parametrize("R,pos", [(8, 2), (8, 15), (3, 9)])
def test_cp_step_stages_vs_fp64(R, pos):
    from qwen_tts import _hip, kernels as Kn
    dev = _dev()
    cp = _CP(dev, seed=21)
    st = cp.st
    if not Kn.cp_step_supported(st.H, st.I, st.Hq, st.Hkv, st.D, st.n_layers, cp.lm.N):
        pytest.skip("qt_cp_step not supported on this device")
    Lmax, g = 18, cp.g
    x = torch.randn(R, st.H, generator=g).to(dev)
    x16 = x.to(torch.bfloat16)
    qkv0 = torch.empty(R, st.qkv_w, device=dev)
    Kn.gemm(x16, st.layers[0].qkv, qkv0, R, st.H, st.qkv_w, rms=True, eps=st.eps)
    kc = [torch.randn(R, st.Hkv, Lmax, st.D, generator=g).to(dev, torch.bfloat16) for _ in st.layers]
    vc = [torch.randn(R, st.Hkv, Lmax, st.D, generator=g).to(dev, torch.bfloat16) for _ in st.layers]
    kc0, vc0 = [k.clone() for k in kc], [v.clone() for v in vc]
    chain = _cp_chain_staged(cp, x.clone(), x16.clone(), qkv0, [k.clone() for k in kc], [v.clone() for v in vc], R,
                             Lmax, pos, dev)
    nws = Kn.cp_step_ws_bytes()
    ws = torch.zeros(nws + int(_hip.lib().qt_cp_step_dbg_bytes()), dtype=torch.uint8, device=dev)
    logits = torch.full((R, cp.lm.N), float("nan"), device=dev)
    Kn.cp_step(st.layers, cp.lm, x, qkv0, R, kc, vc, Lmax, pos, st.cos, st.sin, st.eps, logits, ws)
    torch.cuda.synchronize()
    assert int(ws[:4].view(torch.int32).item()) == 0
    s = _engine_rec(ws, nws, st.n_layers, R)
    eng = {"x_attn": s(0, st.H), "h": s(1, st.I), "x_mlp": s(2, st.H), "att": s(3, st.Hq * st.D),
           "qkv": s(4, st.qkv_w), "logits": logits}
    assert torch.equal(eng["qkv"][0], qkv0)  # layer 0's rows are the input rows
    ee = _stage_errors(cp, eng, x, kc0, vc0, pos, R)
    ce = _stage_errors(cp, chain, x, kc0, vc0, pos, R)
    _assert_ratio(ee, ce, f"cp_step R={R} pos={pos}")


@pytest.mark.parametrize("R", [8, 5])
def test_cp_prefill_stages_vs_fp64(R):
    from qwen_tts import _hip, kernels as Kn
    from qwen_tts.talker import _scratch
    dev = _dev()
    cp = _CP(dev, seed=22)
    st = cp.st
    if not Kn.cp_step_supported(st.H, st.I, st.Hq, st.Hkv, st.D, st.n_layers, cp.lm.N):
        pytest.skip("qt_cp_step not supported on this device")
    Lmax, g = 18, cp.g
    x = torch.randn(2 * R, st.H, generator=g).to(dev)
    kc = [torch.zeros(R, st.Hkv, Lmax, st.D, device=dev, dtype=torch.bfloat16) for _ in st.layers]
    vc = [torch.zeros(R, st.Hkv, Lmax, st.D, device=dev, dtype=torch.bfloat16) for _ in st.layers]
    # the prefill chain (talker._Stack.forward with small_T), stage by stage
    sc = _scratch(2 * R, st, dev, attn_oproj=True)
    xc, x16 = x.clone(), x.to(torch.bfloat16)
    chain = {"qkv": [], "att": [], "x_attn": [], "h": [], "x_mlp": []}
    kcc, vcc = [k.clone() for k in kc], [v.clone() for v in vc]
    for li, L in enumerate(st.layers):
        Kn.gemm(x16, L.qkv, sc["qkv"], 2 * R, st.H, st.qkv_w, rms=True, eps=st.eps)
        chain["qkv"].append(sc["qkv"][:2 * R].clone())
        Kn.small_prefill_attention(sc["qkv"], 2 * R, 2, st.Hq, st.Hkv, st.D, L.q_norm, L.k_norm, st.eps, st.cos, st.sin,
                                   kcc[li], vcc[li], Lmax, sc["att"])
        chain["att"].append(sc["att"][:2 * R].float())
        Kn.gemm(sc["att"], L.o, xc, 2 * R, st.Hq * st.D, st.H, epi=_hip.EPI_ADD, out2=x16)
        chain["x_attn"].append(xc.clone())
        Kn.gemm(x16, L.gu, sc["h"], 2 * R, st.H, st.I, rms=True, eps=st.eps, epi=_hip.EPI_SWIGLU)
        chain["h"].append(sc["h"][:2 * R].float())
        Kn.gemm(sc["h"], L.down, xc, 2 * R, st.I, st.H, epi=_hip.EPI_ADD, out2=x16)
        chain["x_mlp"].append(xc.clone())
    chain["logits"] = torch.empty(R, cp.lm.N, device=dev)
    Kn.gemm(x16.view(-1)[st.H:], cp.lm, chain["logits"], R, 2 * st.H, cp.lm.N, rms=True, eps=st.eps)
    nws = Kn.cp_step_ws_bytes()
    ws = torch.zeros(nws + int(_hip.lib().qt_cp_step_dbg_bytes()), dtype=torch.uint8, device=dev)
    logits = torch.full((R, cp.lm.N), float("nan"), device=dev)
    Kn.cp_prefill(st.layers, cp.lm, x, R, kc, vc, Lmax, st.cos, st.sin, st.eps, logits, ws)
    torch.cuda.synchronize()
    assert int(ws[:4].view(torch.int32).item()) == 0
    s = _engine_rec(ws, nws, st.n_layers, 2 * R)
    eng = {"x_attn": s(0, st.H), "h": s(1, st.I), "x_mlp": s(2, st.H), "att": s(3, st.Hq * st.D),
           "qkv": s(4, st.qkv_w), "logits": logits}
    ee = _stage_errors(cp, eng, x, None, None, 0, R, prefill=True)
    ce = _stage_errors(cp, chain, x, None, None, 0, R, prefill=True)
    _assert_ratio(ee, ce, f"cp_prefill R={R}")


# ---------------------------------------------------------------------------------------------- talker tail
THQ, TD, TQKV, TIMAX = 16, 128, 4096, 6144  # (the stage records' row stride is the largest intermediate size)


class _TL:
    def __init__(self, g, dev, TH, TI):
        from qwen_tts import kernels as Kn
        r = lambda *s: (torch.randn(*s, generator=g) * 0.02)  # noqa: E731
        gam = lambda n: (1 + 0.1 * torch.randn(n, generator=g))  # noqa: E731
        wqkv, gin, wo = r(TQKV, TH), gam(TH), r(TH, THQ * TD)
        wg, wu, gpost, wd = r(TI, TH), r(TI, TH), gam(TH), r(TH, TI)
        self.qkv = Kn.tile_linear(wqkv.to(dev), torch.bfloat16, gamma=gin.to(dev))
        self.o = Kn.tile_linear(wo.to(dev), torch.bfloat16)
        self.gu = Kn.tile_swiglu(wg.to(dev), wu.to(dev), torch.bfloat16, gamma=gpost.to(dev))
        self.down = Kn.tile_linear(wd.to(dev), torch.bfloat16)
        eff = lambda w, gm: (w.to(dev).float() * gm.to(dev).float()[None, :]).to(torch.bfloat16)  # noqa: E731
        self.r_qkv, self.r_o = eff(wqkv, gin), wo.to(dev).to(torch.bfloat16)
        self.r_gate, self.r_up, self.r_down = eff(wg, gpost), eff(wu, gpost), wd.to(dev).to(torch.bfloat16)


@pytest.mark.parametrize("dims", [(2048, 6144), (1024, 3072)])  # the 1.7B / 0.6B talkers
@pytest.mark.parametrize("R", [8, 1])
def test_talker_tail_stages_vs_fp64(R, dims):
    from qwen_tts import _hip, kernels as Kn
    dev = _dev()
    TH, TI = dims
    if not Kn.talker_tail_supported(TH, TI, THQ, TD, TQKV):
        pytest.skip("qt_talker_tail not supported on this device")
    g = torch.Generator().manual_seed(41)
    L, Ln = _TL(g, dev, TH, TI), _TL(g, dev, TH, TI)
    eps = 1e-6
    att = torch.randn(R, THQ * TD, generator=g).to(dev).to(torch.bfloat16)
    x = torch.randn(R, TH, generator=g).to(dev)
    # the chain: o_proj + residual, gate/up + SwiGLU, down + residual, next q/k/v
    xc, x16 = x.clone(), x.to(torch.bfloat16)
    Kn.gemm(att, L.o, xc, R, THQ * TD, TH, epi=_hip.EPI_ADD, out2=x16)
    c_xa = xc.clone()
    h = torch.empty(R, TI, dtype=torch.bfloat16, device=dev)
    Kn.gemm(x16, L.gu, h, R, TH, TI, rms=True, eps=eps, epi=_hip.EPI_SWIGLU)
    Kn.gemm(h, L.down, xc, R, TI, TH, epi=_hip.EPI_ADD, out2=x16)
    c_q = torch.empty(R, TQKV, device=dev)
    Kn.gemm(x16, Ln.qkv, c_q, R, TH, TQKV, rms=True, eps=eps)
    chain = dict(x_attn=c_xa, h=h.float(), x_mlp=xc, qkv=c_q)
    nws = Kn.talker_tail_ws_bytes()
    ws = torch.zeros(nws + int(_hip.lib().qt_talker_tail_dbg_bytes()), dtype=torch.uint8, device=dev)
    xe, qe = x.clone(), torch.full((R, TQKV), float("nan"), device=dev)
    Kn.talker_tail(att, xe, R, L, Ln, qe, eps, ws)
    torch.cuda.synchronize()
    assert int(ws[:4].view(torch.int32).item()) == 0
    d = ws[nws + int(_hip.lib().qt_talker_tail_stamp_bytes()):].view(torch.float32)[:4 * 8 * TIMAX].view(4, 8, TIMAX)
    eng = dict(x_attn=d[0, :R, :TH], h=d[1, :R, :TI], x_mlp=d[2, :R, :TH], qkv=d[3, :R, :TQKV])
    assert torch.equal(eng["x_mlp"], xe) and torch.equal(eng["qkv"], qe)  # the records are the outputs

    def errs(p):
        e = {"x_attn": _rel(p["x_attn"], x.double() + att.double() @ L.r_o.double().T, x)}
        e["h"] = _rel(p["h"], _swiglu_ref(p["x_attn"], L.r_gate, L.r_up, eps))
        e["x_mlp"] = _rel(p["x_mlp"], p["x_attn"].double() + _bf(p["h"]) @ L.r_down.double().T, p["x_attn"])
        e["qkv"] = _rel(p["qkv"], _rms_lin(p["x_mlp"], Ln.r_qkv, eps))
        return e
    ee, ce = errs(eng), errs(chain)
    print(f"\n  talker_tail H={TH} R={R} (engine / chain error vs fp64): " +
          "  ".join(f"{k} {ee[k]:.2e}/{ce[k]:.2e}" for k in ee))
    for k in ee:
        assert ee[k] < 1e-2, (k, ee[k])
        assert ee[k] <= RATIO * ce[k] + FLOOR, (k, ee[k], ce[k])
