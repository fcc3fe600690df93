"""qt_talker_tail (csrc/talker_tail.hip): the part of a 1.7B talker decoder layer after its attention -- o_proj +
residual, gate/up + SwiGLU, down + residual, the next layer's q/k/v -- in one persistent launch, against the launch
chain of qt_gemm decode GEMVs it replaces (_Stack.forward, M:961-1012) on the same random weights and rows."""
import pytest
import torch

pytestmark = pytest.mark.gpu

H, I, HQ, D, QKV = 2048, 6144, 16, 128, 4096


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


class _L:
    """The tiled weights of one talker layer (as talker._Layer holds them)."""

    def __init__(self, g, dev):
        from qwen_tts import kernels as Kn
        r = lambda *s: (torch.randn(*s, generator=g) * 0.02).to(dev)  # noqa: E731
        gam = lambda n: (1 + 0.1 * torch.randn(n, generator=g)).to(dev)  # noqa: E731
        self.qkv = Kn.tile_linear(r(QKV, H), torch.bfloat16, gamma=gam(H))
        self.o = Kn.tile_linear(r(H, HQ * D), torch.bfloat16)
        self.gu = Kn.tile_swiglu(r(I, H), r(I, H), torch.bfloat16, gamma=gam(H))
        self.down = Kn.tile_linear(r(H, I), torch.bfloat16)


_CACHE = {}


def _layers(dev):
    if "L" not in _CACHE:
        g = torch.Generator().manual_seed(11)
        _CACHE["L"] = (_L(g, dev), _L(g, dev))
    return _CACHE["L"]


def _chain(att, x, L, Ln, R, eps):
    from qwen_tts import _hip, kernels as Kn
    x = x.clone()
    x16 = x.to(torch.bfloat16)
    Kn.gemm(att, L.o, x, R, HQ * D, H, epi=_hip.EPI_ADD, out2=x16)
    h = torch.empty(R, I, dtype=torch.bfloat16, device=x.device)
    Kn.gemm(x16, L.gu, h, R, H, I, rms=True, eps=eps, epi=_hip.EPI_SWIGLU)
    Kn.gemm(h, L.down, x, R, I, H, epi=_hip.EPI_ADD, out2=x16)
    qkv = None
    if Ln is not None:
        qkv = torch.empty(R, QKV, device=x.device)
        Kn.gemm(x16, Ln.qkv, qkv, R, H, QKV, rms=True, eps=eps)
    return x, qkv


def _rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm())


def _inputs(R, dev, seed=3):
    g = torch.Generator().manual_seed(seed)
    att = torch.randn(R, HQ * D, generator=g).to(dev).to(torch.bfloat16)
    x = torch.randn(R, H, generator=g).to(dev)
    return att, x


def test_talker_tail_supported_here():
    from qwen_tts import kernels as Kn
    _dev()
    assert Kn.talker_tail_supported(H, I, HQ, D, QKV)


@pytest.mark.parametrize("R", [1, 3, 8])
def test_talker_tail_matches_chain(R):
    from qwen_tts import kernels as Kn
    dev = _dev()
    L, Ln = _layers(dev)
    eps = 1e-6
    att, x = _inputs(R, dev)
    xr, qr = _chain(att, x, L, Ln, R, eps)
    ws = torch.zeros(Kn.talker_tail_ws_bytes(), dtype=torch.uint8, device=dev)
    outs = []
    for _ in range(3):
        xe = x.clone()
        qe = torch.full((R, QKV), float("nan"), device=dev)
        Kn.talker_tail(att, xe, R, L, Ln, qe, eps, ws)
        torch.cuda.synchronize()
        assert int(ws[:4].view(torch.int32).item()) == 0
        outs.append((xe, qe))
    xe, qe = outs[0]
    print(f"\n  R={R}: x rel {_rel(xe, xr):.3e}, qkv rel {_rel(qe, qr):.3e}")
    assert torch.isfinite(qe).all()
    assert _rel(xe, xr) < 2e-3
    assert _rel(qe, qr) < 2e-2
    for xo, qo in outs[1:]:  # deterministic (fixed reduction orders)
        assert torch.equal(xo, xe) and torch.equal(qo, qe)


def test_talker_tail_last_layer_and_many_launches():
    """Without a next layer only x is produced (qkv untouched); 30 launches alternating both forms on one workspace
    (the launch counter advances, nothing is reset) reproduce the first results."""
    from qwen_tts import kernels as Kn
    dev = _dev()
    L, Ln = _layers(dev)
    R, eps = 8, 1e-6
    att, x = _inputs(R, dev, seed=5)
    xr, _ = _chain(att, x, L, None, R, eps)
    ws = torch.zeros(Kn.talker_tail_ws_bytes(), dtype=torch.uint8, device=dev)
    first = None
    for it in range(30):
        xe = x.clone()
        qe = torch.full((R, QKV), 7.0, device=dev)
        nxt = Ln if it % 2 else None
        Kn.talker_tail(att, xe, R, L, nxt, qe, eps, ws)
        torch.cuda.synchronize()
        if nxt is None:
            assert bool((qe == 7.0).all())
            assert _rel(xe, xr) < 2e-3
            if first is None:
                first = xe
            assert torch.equal(xe, first)
    assert int(ws[4:8].view(torch.int32).item()) == 30
    assert int(ws[:4].view(torch.int32).item()) == 0
