"""qt_talker_tail (csrc/talker_tail.hip): the part of a talker decoder layer after its attention -- o_proj + residual,
gate/up + SwiGLU, down + residual, the next layer's q/k/v -- in one persistent launch, against the launch chain of
qt_gemm decode GEMVs it replaces (_Stack.forward, M:961-1012) on the same random weights and rows, at both talkers'
dims from their configs: 1.7B (hidden 2048, intermediate 6144: 256 workgroups) and 0.6B (1024, 3072: 128)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

H, I, HQ, D, QKV = 2048, 6144, 16, 128, 4096
DIMS = [(2048, 6144), (1024, 3072)]  # (hidden, intermediate) of the 1.7B / 0.6B talkers


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


class _L:
    """The tiled weights of one talker layer (as talker._Layer holds them)."""

    def __init__(self, g, dev, Hd=H, Id=I):
        from qwen_tts import kernels as Kn
        r = lambda *s: (torch.randn(*s, generator=g) * 0.02).to(dev)  # noqa: E731
        gam = lambda n: (1 + 0.1 * torch.randn(n, generator=g)).to(dev)  # noqa: E731
        self.qkv = Kn.tile_linear(r(QKV, Hd), torch.bfloat16, gamma=gam(Hd))
        self.o = Kn.tile_linear(r(Hd, HQ * D), torch.bfloat16)
        self.gu = Kn.tile_swiglu(r(Id, Hd), r(Id, Hd), torch.bfloat16, gamma=gam(Hd))
        self.down = Kn.tile_linear(r(Hd, Id), torch.bfloat16)
        self.H, self.I = Hd, Id


_CACHE = {}


def _layers(dev, Hd=H, Id=I):
    if (Hd, Id) not in _CACHE:
        g = torch.Generator().manual_seed(11)
        _CACHE[(Hd, Id)] = (_L(g, dev, Hd, Id), _L(g, dev, Hd, Id))
    return _CACHE[(Hd, Id)]


def _chain(att, x, L, Ln, R, eps):
    from qwen_tts import _hip, kernels as Kn
    Hd, Id = L.H, L.I
    x = x.clone()
    x16 = x.to(torch.bfloat16)
    Kn.gemm(att, L.o, x, R, HQ * D, Hd, epi=_hip.EPI_ADD, out2=x16)
    h = torch.empty(R, Id, dtype=torch.bfloat16, device=x.device)
    Kn.gemm(x16, L.gu, h, R, Hd, Id, rms=True, eps=eps, epi=_hip.EPI_SWIGLU)
    Kn.gemm(h, L.down, x, R, Id, Hd, epi=_hip.EPI_ADD, out2=x16)
    qkv = None
    if Ln is not None:
        qkv = torch.empty(R, QKV, device=x.device)
        Kn.gemm(x16, Ln.qkv, qkv, R, Hd, QKV, rms=True, eps=eps)
    return x, qkv


def _rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm())


def _inputs(R, dev, seed=3, Hd=H):
    g = torch.Generator().manual_seed(seed)
    att = torch.randn(R, HQ * D, generator=g).to(dev).to(torch.bfloat16)
    x = torch.randn(R, Hd, generator=g).to(dev)
    return att, x


def test_talker_tail_supported_here():
    from qwen_tts import kernels as Kn
    _dev()
    for Hd, Id in DIMS:
        assert Kn.talker_tail_supported(Hd, Id, HQ, D, QKV), (Hd, Id)
    assert not Kn.talker_tail_supported(1536, 4608, HQ, D, QKV)  # a shape it has no instance for


@pytest.mark.parametrize("dims", DIMS)
@pytest.mark.parametrize("R", [1, 3, 8])
def test_talker_tail_matches_chain(R, dims):
    from qwen_tts import kernels as Kn
    dev = _dev()
    L, Ln = _layers(dev, *dims)
    eps = 1e-6
    att, x = _inputs(R, dev, Hd=dims[0])
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
    print(f"\n  H={dims[0]} R={R}: x rel {_rel(xe, xr):.3e}, qkv rel {_rel(qe, qr):.3e}")
    assert torch.isfinite(qe).all()
    assert _rel(xe, xr) < 2e-4  # measured <= 3.6e-5 (summation order; fp32 residual)
    assert _rel(qe, qr) < 1e-3  # measured <= 2.3e-4 (x16 rounding flips of the bf16 operand)
    for xo, qo in outs[1:]:  # deterministic (fixed reduction orders)
        assert torch.equal(xo, xe) and torch.equal(qo, qe)


@pytest.mark.parametrize("dims", DIMS)
def test_talker_tail_last_layer_and_many_launches(dims):
    """Without a next layer only x is produced (qkv untouched); 30 launches alternating both forms on one workspace
    (the launch counter advances, nothing is reset) reproduce the first results."""
    from qwen_tts import kernels as Kn
    dev = _dev()
    L, Ln = _layers(dev, *dims)
    R, eps = 8, 1e-6
    att, x = _inputs(R, dev, seed=5, Hd=dims[0])
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
            assert _rel(xe, xr) < 2e-4
            if first is None:
                first = xe
            assert torch.equal(xe, first)
    assert int(ws[4:8].view(torch.int32).item()) == 30
    assert int(ws[:4].view(torch.int32).item()) == 0
