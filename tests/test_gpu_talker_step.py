"""qt_talker_step (csrc/talker_step.hip): every decoder layer of a 1.7B talker decode step -- q/k/v, q/k norm + RoPE +
KV append + attention, o_proj, gate/up + SwiGLU, down -- in one persistent launch, against the launch chain
(_Stack.forward(decode=True), M:1430-1480) on the same random weights, ragged rows (different cache lengths, left
pads, cache batch entries) and caches."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


_ST = {}


def _stack(dev, n_layers=28):
    """The talker backbone (1.7B dims, seeded random weights, n_layers layers)."""
    if n_layers not in _ST:
        import os
        from qwen_tts.talker import _Stack
        from qwen_tts.weights import read_json, resolve_path, synthetic, talker_specs
        _ST.clear()
        cfg = read_json(os.path.join(resolve_path("synthetic:1.7b-customvoice"), "config.json"))
        tc = dict(cfg["talker_config"], num_hidden_layers=n_layers)
        pre = "talker.model"
        specs = [(n, s) for n, s in talker_specs(cfg) if n == pre + ".norm.weight" or
                 (n.startswith(pre + ".layers.") and int(n.split(".")[3]) < n_layers)]
        W = synthetic(specs, dev)
        _ST[n_layers] = _Stack(W, pre, tc, torch.bfloat16, dev, 4096)
    return _ST[n_layers]


def _rows(B, dev, seed):
    g = torch.Generator().manual_seed(seed)
    kv_pos = torch.randint(60, 300, (B,), generator=g)
    row_start = torch.where(torch.rand(B, generator=g) < 0.5, torch.randint(0, 40, (B,), generator=g), 0)
    rope_pos = kv_pos - row_start
    row_batch = torch.randperm(B, generator=g)
    i32 = lambda t: t.to(torch.int32).to(dev)  # noqa: E731
    return {"rope_pos": i32(rope_pos), "kv_pos": i32(kv_pos), "row_start": i32(row_start),
            "row_batch": i32(row_batch), "nsplit": 1}


def _caches(st, B, Lmax, dev, seed):
    g = torch.Generator().manual_seed(seed)
    kc = [(torch.randn(B, st.Hkv, Lmax, st.D, generator=g) * 0.5).to(dev).to(torch.bfloat16) for _ in st.layers]
    vc = [(torch.randn(B, st.Hkv, Lmax, st.D, generator=g) * 0.5).to(dev).to(torch.bfloat16) for _ in st.layers]
    return kc, vc


def _rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm())


def _run(st, B, xe, ke, ve, Lmax, meta, ws, per_layer):
    """The engine over all layers: one launch, or one launch per layer chained through q/k/v rows (layer 0's from
    the q/k/v GEMV on the bf16 input rows, as the frame issues it)."""
    from qwen_tts import kernels as Kn
    tab = Kn.talker_step_table(st.layers, ke, ve, xe.device)
    args = (B, xe, Lmax, st.cos, st.sin, meta["rope_pos"], meta["kv_pos"], meta["row_start"], meta["row_batch"],
            st.eps, ws)
    if not per_layer:
        Kn.talker_step(tab, st.n_layers, *args)
        return
    if per_layer == "att":  # layer 0's q/k/v + attention on the chain, then per layer: o_proj .. next attention
        q0 = torch.empty(B, st.qkv_w, device=xe.device)
        Kn.gemm(xe.to(torch.bfloat16), st.layers[0].qkv, q0, B, st.H, st.qkv_w, rms=True, eps=st.eps)
        a = [torch.empty(B, st.Hq * st.D, dtype=torch.bfloat16, device=xe.device) for _ in range(2)]
        L0 = st.layers[0]
        Kn.decode_attention(q0, B, st.Hq, st.Hkv, st.D, L0.q_norm, L0.k_norm, st.eps, st.cos, st.sin, meta["rope_pos"],
                            meta["row_batch"], meta["kv_pos"], meta["row_start"], ke[0], ve[0], Lmax, a[0])
        for li in range(st.n_layers):
            Kn.talker_step(tab, 1, *args, first_layer=li, total_layers=st.n_layers, att_in=a[li % 2],
                           att_out=a[(li + 1) % 2] if li + 1 < st.n_layers else None)
        return
    q = [torch.empty(B, st.qkv_w, device=xe.device) for _ in range(2)]
    Kn.gemm(xe.to(torch.bfloat16), st.layers[0].qkv, q[0], B, st.H, st.qkv_w, rms=True, eps=st.eps)
    for li in range(st.n_layers):
        Kn.talker_step(tab, 1, *args, first_layer=li, total_layers=st.n_layers, qkv_in=q[li % 2],
                       qkv_out=q[(li + 1) % 2] if li + 1 < st.n_layers else None)


@pytest.mark.parametrize("B,n_layers,per_layer", [(8, 28, False), (3, 4, False), (1, 2, False), (8, 28, True),
                                                  (3, 4, True), (8, 28, "att"), (3, 4, "att")])
def test_talker_step_matches_chain(B, n_layers, per_layer):
    from qwen_tts import kernels as Kn
    from qwen_tts.talker import _scratch
    dev = _dev()
    st = _stack(dev, n_layers)
    assert Kn.talker_step_supported(st.H, st.I, st.Hq, st.Hkv, st.D, st.n_layers)
    Lmax = 320
    meta = _rows(B, dev, 7 + B)
    kc, vc = _caches(st, B, Lmax, dev, 3)
    g = torch.Generator().manual_seed(11)
    x0 = torch.randn(B, st.H, generator=g).to(dev)
    # the chain
    xr = x0.clone()
    x16 = xr.to(torch.bfloat16)
    kr, vr = [k.clone() for k in kc], [v.clone() for v in vc]
    st.forward(xr, B, meta, (kr, vr), _scratch(B, st, dev), Lmax, Lmax, decode=True, x16=x16)
    # the engine, twice on one workspace (the second from the same inputs)
    ws = torch.zeros(Kn.talker_step_ws_bytes(), dtype=torch.uint8, device=dev)
    outs = []
    for _ in range(2):
        xe = x0.clone()
        ke, ve = [k.clone() for k in kc], [v.clone() for v in vc]
        _run(st, B, xe, ke, ve, Lmax, meta, ws, per_layer)
        torch.cuda.synchronize()
        assert int(ws[:4].view(torch.int32).item()) == 0, "hand-off flag"
        outs.append((xe, ke, ve))
    xe, ke, ve = outs[0]
    rel = _rel(xe, xr)
    kv_pos, rb = meta["kv_pos"].cpu(), meta["row_batch"].cpu()
    knew = torch.stack([ke[l][rb[r], :, kv_pos[r]] for l in range(n_layers) for r in range(B)]).float()
    kref = torch.stack([kr[l][rb[r], :, kv_pos[r]] for l in range(n_layers) for r in range(B)]).float()
    print(f"\n  B={B} L={n_layers} per_layer={per_layer}: x rel {rel:.3e}, appended keys rel {_rel(knew, kref):.3e}")
    assert torch.isfinite(xe).all()
    assert rel < 2e-2
    assert _rel(knew, kref) < 2e-2
    # everything but the appended slots is untouched
    for l in range(n_layers):
        mk = torch.ones(B, Lmax, dtype=torch.bool)
        mk[rb, kv_pos] = False
        assert torch.equal(ke[l].permute(0, 2, 1, 3)[mk.to(dev)], kc[l].permute(0, 2, 1, 3)[mk.to(dev)])
    x2, k2, _ = outs[1]
    assert torch.equal(x2, xe) and all(torch.equal(a, b) for a, b in zip(k2, ke))  # deterministic
    assert int(ws[4:8].view(torch.int32).item()) == 2 * (n_layers if per_layer else 1)
