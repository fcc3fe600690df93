"""GPU parity of the voice-clone front end through the HIP C-ABI library.

* Kernel units (qt_pad_time, qt_layernorm, qt_rvq_encode, qt_time_stats, qt_mel_logmag, qt_scale_add,
  qt_bcast_rows, GEMM ELU prologue / ReLU / sigmoid / tanh∘ReLU epilogues, the polyphase strided conv) against
  plain torch fp32 on seeded inputs.
* Tokenizer encoder (Mimi) against the reference's codes (tests/golden/frontend_*.npz): fp32 mode must be
  bit-exact except where the reference's own choice is a near-tie (relative gap between the two nearest
  codewords < 1e-3, measured by the fp64 oracle) -- after such a tie the rest of that frame's residual chain
  legitimately diverges.  bf16 mode: >= 95% of semantic (cb0) codes and >= 90% of all codes agree
  (measured: 100% / 99.1% tiny, 100% / 97.4% 1.7B dims).
* Speaker encoder: log-mel |diff| <= 1e-3, x-vector relative L2 error <= 1e-3 (fp32), <= 5e-2 (bf16).
* End to end: create_voice_clone_prompt / generate_voice_clone on the tiny Base preset.
"""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


# ------------------------------------------------------------------------------------------ kernels
@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_pad_time_modes(mode, dtype):
    from qwen_tts import kernels as Kn
    dev = _dev()
    g = torch.Generator().manual_seed(mode)
    B, T, C, l, r = 2, 9, 5, 3, 2
    x = torch.randn(B, T, C, generator=g).to(dtype)
    x2 = torch.randn(B, T, C, generator=g).to(dtype)
    tt = T + l + r + 4
    out = torch.full((B, tt, C), 7.0, dtype=dtype, device=dev)
    Kn.pad_time(x.to(dev), B, T, C, l, r, mode, out, t_total=tt, x2=x2.to(dev))
    s = (x.float() + x2.float()).transpose(1, 2)
    pm = {0: "constant", 1: "reflect", 2: "replicate"}[mode]
    ref = F.pad(s, (l, r), mode=pm).transpose(1, 2)
    ref = torch.cat([ref, torch.zeros(B, 4, C)], 1).to(dtype)
    if mode == 0:
        ref[:, :l] = 0
        ref[:, l + T:] = 0
    torch.testing.assert_close(out.cpu(), ref, atol=0, rtol=0) if dtype == torch.float32 else \
        torch.testing.assert_close(out.cpu().float(), ref.float(), atol=1e-2, rtol=1e-2)


def test_zero_tail_and_bcast_scale_add():
    from qwen_tts import kernels as Kn
    dev = _dev()
    g = torch.Generator().manual_seed(5)
    x = torch.randn(3, 10, 6, generator=g).to(dev)
    y = x.clone()
    Kn.zero_tail(y, 3, 10, 7, 6)
    ref = x.clone()
    ref[:, 7:] = 0
    assert torch.equal(y, ref)
    v = torch.randn(3, 8, generator=g).to(dev)
    o = torch.zeros(3, 10, 12, device=dev)
    Kn.bcast_rows(v, 3, 10, 8, o[:, :, 4:], ldo=12)
    assert torch.equal(o[:, :, 4:], v[:, None, :].expand(3, 10, 8)) and torch.equal(o[:, :, :4], torch.zeros(3, 10, 4, device=dev))
    s = torch.rand(3, 6, generator=g).to(dev)
    res = torch.randn(3, 10, 6, generator=g).to(dev)
    out = torch.empty_like(x)
    Kn.scale_add(x, s, res, 3, 10, 6, out)
    torch.testing.assert_close(out, x * s[:, None, :] + res)


@pytest.mark.parametrize("M,N", [(37, 64), (5, 512), (130, 1000)])
def test_layernorm(M, N):
    from qwen_tts import kernels as Kn
    dev = _dev()
    g = torch.Generator().manual_seed(N)
    x = torch.randn(M, N, generator=g) * 3 + 1
    w, b = 1 + 0.1 * torch.randn(N, generator=g), 0.1 * torch.randn(N, generator=g)
    out = torch.empty(M, N, device=dev)
    Kn.layernorm(x.to(dev), w.to(dev), b.to(dev), 1e-5, out, M, N)
    torch.testing.assert_close(out.cpu(), F.layer_norm(x, (N,), w, b, 1e-5), atol=2e-5, rtol=2e-5)


@pytest.mark.parametrize("act", [3, 4, 5])
def test_gemm_new_activations(act):
    from qwen_tts import kernels as Kn
    dev = _dev()
    g = torch.Generator().manual_seed(act)
    M, N, K = 40, 48, 64
    W, A, b = torch.randn(N, K, generator=g) * 0.2, torch.randn(M, K, generator=g), torch.randn(N, generator=g) * 0.1
    t = Kn.tile_linear(W.to(dev), torch.float32, b.to(dev))
    for m in (M, 3):  # tiled GEMM and the decode GEMV path
        out = torch.empty(m, N, device=dev)
        Kn.gemm(A[:m].to(dev), t, out, m, K, N, act=act)
        z = A[:m] @ W.T + b
        ref = {3: torch.relu(z), 4: torch.sigmoid(z), 5: torch.tanh(torch.relu(z))}[act]
        torch.testing.assert_close(out.cpu(), ref, atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("cin,cout,k,T", [(32, 16, 3, 200), (64, 128, 1, 150), (16, 32, 7, 300)])
def test_gemm_conv_elu_prologue(dtype, cin, cout, k, T):
    from qwen_tts import kernels as Kn, _hip
    dev = _dev()
    g = torch.Generator().manual_seed(cin * k)
    B = 2
    w, b = torch.randn(cout, cin, k, generator=g) * 0.2, torch.randn(cout, generator=g) * 0.1
    x = torch.randn(B, T, cin, generator=g)
    t = Kn.tile_conv(w.to(dev), b.to(dev), dtype)
    out = torch.empty(B * T, cout, device=dev)
    Kn.gemm(x.to(dev), t, out, B * T, cin, cout, conv=(T, T, -(k - 1), 1), a_act=_hip.AACT_ELU)
    xa = F.elu(x)
    if dtype == torch.bfloat16:
        xa = xa.to(dtype).float()
    ref = F.conv1d(F.pad(xa.transpose(1, 2), (k - 1, 0)), w.to(dtype).float(), b).transpose(1, 2).reshape(B * T, cout)
    tol = 1e-4 if dtype == torch.float32 else 2e-2
    torch.testing.assert_close(out.cpu(), ref, atol=tol, rtol=tol)


@pytest.mark.parametrize("r,C,L", [(4, 16, 803), (5, 32, 400), (8, 8, 1001), (2, 64, 77)])
def test_polyphase_strided_conv(r, C, L):
    """MimiConv1d(kernel 2r, stride r, causal, zero extra padding) as the encoder runs it: zero the tail of a
    longer buffer, read it as [Tp/r][r*C] and run a 2-tap conv with the relaid-out weight."""
    from qwen_tts import kernels as Kn, _hip
    from qwen_tts.encoder import _polyphase_weight, _tile_taps
    dev = _dev()
    g = torch.Generator().manual_seed(r * C)
    B = 2
    Tp = -(-L // r) * r + 2 * r
    w, b = torch.randn(2 * C, C, 2 * r, generator=g) * 0.1, torch.randn(2 * C, generator=g) * 0.1
    x = torch.randn(B, Tp, C, generator=g)
    xd = x.to(dev).reshape(B * Tp, C).clone()
    Kn.zero_tail(xd, B, Tp, L, C)
    t = _tile_taps(_polyphase_weight(w.to(dev), r), b.to(dev), torch.float32, r * C)
    Tn = Tp // r
    out = torch.empty(B * Tn, 2 * C, device=dev)
    Kn.gemm(xd, t, out, B * Tn, r * C, 2 * C, conv=(Tn, Tn, -1, 1), a_act=_hip.AACT_ELU)
    xs = F.elu(x[:, :L]).transpose(1, 2)
    extra = -(-L // r) * r - L
    ref = F.conv1d(F.pad(xs, (r, extra)), w, b, stride=r).transpose(1, 2)
    nv = ref.shape[1]
    torch.testing.assert_close(out.view(B, Tn, 2 * C)[:, :nv].cpu(), ref, atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize("D,cb,Q,R", [(32, 2048, 15, 21), (256, 2048, 3, 8), (24, 320, 4, 5), (256, 2048, 2, 77)])
def test_rvq_encode_nearest_codeword(D, cb, Q, R):
    from qwen_tts import kernels as Kn
    dev = _dev()
    g = torch.Generator().manual_seed(D + Q)
    tab = torch.randn(Q, cb, D, generator=g) / torch.rand(Q, cb, 1, generator=g).clamp(min=0.3)
    x = torch.randn(R, D, generator=g) * 2
    codes = torch.full((R, Q + 1), -1, dtype=torch.int32, device=dev)
    Kn.rvq_encode(x.to(dev), D, tab.to(dev), tab.transpose(1, 2).contiguous().to(dev), Q, cb, D, R, codes[:, 1:], Q + 1)
    res = x.double()
    ref = []
    for q in range(Q):
        d = ((res[:, None, :] - tab[q].double()[None]) ** 2).sum(-1)
        i = d.argmin(-1)
        ref.append(i)
        res = res - tab[q].double()[i]
    assert torch.equal(codes[:, 1:].cpu().long(), torch.stack(ref, 1))
    assert (codes[:, 0] == -1).all()


def test_time_stats_and_mel():
    from qwen_tts import kernels as Kn
    dev = _dev()
    g = torch.Generator().manual_seed(11)
    B, T, C = 2, 37, 70
    x = torch.randn(B, T, C, generator=g)
    lg = torch.randn(B, T, C, generator=g) * 3
    m = torch.empty(B, C, device=dev)
    s = torch.empty(B, C, device=dev)
    Kn.time_stats(x.to(dev), B, T, C, m, s)
    torch.testing.assert_close(m.cpu(), x.mean(1), atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(s.cpu(), x.var(1, unbiased=False).clamp(min=1e-12).sqrt(), atol=1e-5, rtol=1e-5)
    Kn.time_stats(x.to(dev), B, T, C, m, s, logits=lg.to(dev))
    a = torch.softmax(lg, 1)
    mr = (a * x).sum(1)
    torch.testing.assert_close(m.cpu(), mr, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(s.cpu(), (a * (x - mr[:, None]) ** 2).sum(1).clamp(min=1e-12).sqrt(), atol=1e-5, rtol=1e-5)
    Fn, nb, nm = 9, 513, 128
    spec = torch.randn(Fn, 2 * nb, generator=g)
    basis = torch.rand(nm, nb, generator=g) * 0.01
    out = torch.empty(Fn, nm, device=dev)
    Kn.mel_logmag(spec.to(dev), 2 * nb, Fn, nb, basis.to(dev), nm, out)
    mag = torch.sqrt(spec.view(Fn, nb, 2).pow(2).sum(-1) + 1e-9)
    torch.testing.assert_close(out.cpu(), torch.log(torch.clamp(mag @ basis.T, min=1e-5)), atol=1e-5, rtol=1e-5)


# ------------------------------------------------------------------------------------------ golden (reference)
CASES = [("tiny-base", "tiny", "frontend_tiny.npz"), ("1.7b-base", "full", "frontend_full.npz")]


def _encoder(preset, dtype):
    from oracle import load_preset, synth_param
    from oracle.encoder import encoder_param_specs
    from qwen_tts.encoder import TokenizerEncoder
    _, ccfg = load_preset(preset)
    W = {n: synth_param(n, s) for n, s in encoder_param_specs(ccfg)}
    return ccfg, W, TokenizerEncoder(ccfg, W, dtype=dtype, device=_dev())


def _check_codes(got, gold, margins, tol=1e-3):
    """Bit-exact codes, except that a frame may diverge from the first near-tie of the reference on."""
    ties = 0
    for f in range(gold.shape[0]):
        for q in range(gold.shape[1]):
            if got[f, q] != gold[f, q]:
                assert margins[f, q] < tol, (f, q, got[f, q], gold[f, q], margins[f, q])
                ties += 1
                break
    return ties


@pytest.mark.parametrize("preset,kind,fname", CASES)
def test_encoder_matches_reference_fp32(preset, kind, fname):
    from cases import frontend_cases, ref_audio
    from oracle.encoder import EncoderOracle
    z = np.load(os.path.join(GOLD, fname))
    ccfg, W, enc = _encoder(preset, "fp32")
    eo = EncoderOracle(ccfg, W)
    ties = 0
    for key, lens in frontend_cases()[kind]["enc"].items():
        wavs = [ref_audio(n, 1000 + 10 * i + n % 97) for i, n in enumerate(lens)]
        got = enc.encode([torch.from_numpy(w) for w in wavs])
        L = max(lens)
        xb = torch.zeros(len(wavs), L)
        for i, w in enumerate(wavs):
            xb[i, :len(w)] = torch.from_numpy(w)
        marg = eo.margins(eo.embeddings(xb), 16)  # [B, 16, T12]
        for j, c in enumerate(got):
            gold = z[f"enc/{key}/codes{j}"]
            assert tuple(c.shape) == gold.shape, (key, j)
            ties += _check_codes(c.cpu().numpy(), gold, marg[j, :, :gold.shape[0]].T.numpy())
    assert ties <= 2


@pytest.mark.parametrize("preset,kind,fname", CASES)
def test_encoder_bf16_tracks_reference(preset, kind, fname):
    from cases import frontend_cases, ref_audio
    z = np.load(os.path.join(GOLD, fname))
    _, _, enc = _encoder(preset, "bf16")
    n0 = a0 = n = a = 0
    for key, lens in frontend_cases()[kind]["enc"].items():
        wavs = [ref_audio(nn, 1000 + 10 * i + nn % 97) for i, nn in enumerate(lens)]
        for j, c in enumerate(enc.encode([torch.from_numpy(w) for w in wavs])):
            gold = z[f"enc/{key}/codes{j}"]
            c = c.cpu().numpy()
            assert c.shape == gold.shape
            n0 += gold.shape[0]
            a0 += int((c[:, 0] == gold[:, 0]).sum())
            n += gold.size
            a += int((c == gold).sum())
    print(f"bf16 code agreement {preset}: cb0 {a0 / n0:.3f} all {a / n:.3f}")
    assert a0 / n0 >= 0.95 and a / n >= 0.9, (a0 / n0, a / n)


def _speaker(preset, dtype):
    from oracle import load_preset, synth_param
    from oracle.speaker import speaker_param_specs
    from qwen_tts.speaker import SpeakerEncoder
    cfg, _ = load_preset(preset)
    W = {n: synth_param(n, s) for n, s in speaker_param_specs(cfg)}
    return SpeakerEncoder(cfg, W, dtype=dtype, device=_dev())


@pytest.mark.parametrize("preset,kind,fname", CASES)
@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_speaker_encoder_matches_reference(preset, kind, fname, dtype):
    from cases import frontend_cases, ref_audio
    z = np.load(os.path.join(GOLD, fname))
    se = _speaker(preset, dtype)
    for j, n in enumerate(frontend_cases()[kind]["spk"]):
        w = ref_audio(n, 2000 + j)
        mel = se.mel(torch.from_numpy(w).to(se.dev))
        np.testing.assert_allclose(mel.cpu().numpy(), z[f"spk/{j}/mel"], atol=1e-3, rtol=0)
        emb = se.embed(w).cpu().numpy()
        ref = z[f"spk/{j}/emb"]
        rel = np.linalg.norm(emb - ref) / np.linalg.norm(ref)
        assert rel < (1e-3 if dtype == "fp32" else 5e-2), rel


def test_speaker_encoder_rejects_short_audio():
    se = _speaker("tiny-base", "fp32")
    with pytest.raises(ValueError):
        se.embed(np.zeros(300, np.float32))


# ------------------------------------------------------------------------------------------ end to end
@pytest.fixture(scope="module")
def tiny_base():
    from oracle import load_preset, synth_param, synth_state_dict, talker_param_specs, codec_param_specs
    from oracle.encoder import encoder_param_specs
    from oracle.speaker import speaker_param_specs
    from qwen_tts import Qwen3TTSModel
    _dev()
    cfg, ccfg = load_preset("tiny-base")
    W = {k: torch.from_numpy(v) for k, v in synth_state_dict(talker_param_specs(cfg) + speaker_param_specs(cfg)).items()}
    CW = {k: torch.from_numpy(v) for k, v in synth_state_dict(codec_param_specs(ccfg) + encoder_param_specs(ccfg)).items()}
    return Qwen3TTSModel.from_pretrained("synthetic:tiny-base", dtype=torch.float32, weights=W, codec_weights=CW)


def test_tokenizer_encode_api(tiny_base):
    """Qwen3TTSTokenizer.encode input forms (Z:208-257): ndarray + sr, list of ndarrays, WAV base64; the
    codes round-trip shape through decode."""
    import base64
    import io
    import wave
    from cases import ref_audio
    tok = tiny_base.model.speech_tokenizer
    w = ref_audio(31234, 1000 + 31234 % 97)
    z = np.load(os.path.join(GOLD, "frontend_tiny.npz"))
    out = tok.encode(w, sr=24000)
    np.testing.assert_array_equal(out.audio_codes[0].cpu().numpy(), z["enc/single/codes0"])
    out2 = tok.encode([w], sr=24000, return_dict=False)
    assert torch.equal(out2[0][0], out.audio_codes[0])
    pcm = np.clip(np.round(w * 32767), -32768, 32767).astype("<i2")
    buf = io.BytesIO()
    with wave.open(buf, "wb") as f:
        f.setnchannels(1)
        f.setsampwidth(2)
        f.setframerate(24000)
        f.writeframes(pcm.tobytes())
    b64 = "data:audio/wav;base64," + base64.b64encode(buf.getvalue()).decode()  # W:188-194 heuristic
    c16 = tok.encode(b64).audio_codes[0]
    assert c16.shape == out.audio_codes[0].shape
    with pytest.raises(ValueError):
        tok.encode(w)  # numpy input needs sr
    wavs, sr = tok.decode(out)
    assert sr == 24000 and wavs[0].ndim == 1


def test_voice_clone_prompt_and_generate(tiny_base):
    from cases import ref_audio
    from oracle import load_preset, synth_param
    from oracle.speaker import SpeakerOracle, speaker_param_specs
    tts = tiny_base
    w = ref_audio(31234, 1000 + 31234 % 97)
    z = np.load(os.path.join(GOLD, "frontend_tiny.npz"))
    items = tts.create_voice_clone_prompt((w, 24000), ref_text="a reference transcript")
    assert len(items) == 1 and items[0].icl_mode and not items[0].x_vector_only_mode
    np.testing.assert_array_equal(items[0].ref_code.cpu().numpy(), z["enc/single/codes0"])
    cfg, _ = load_preset("tiny-base")
    so = SpeakerOracle(cfg, {n: synth_param(n, s) for n, s in speaker_param_specs(cfg)})
    ref = so.embed(w).numpy()
    got = items[0].ref_spk_embedding.cpu().numpy()
    assert np.linalg.norm(got - ref) / np.linalg.norm(ref) < 1e-3
    kw = dict(max_new_tokens=6, do_sample=False, subtalker_dosample=False)
    wa, sr = tts.generate_voice_clone("hello there", language="English", voice_clone_prompt=items, **kw)
    wb, _ = tts.generate_voice_clone("hello there", language="English", ref_audio=(w, 24000),
                                     ref_text="a reference transcript", **kw)
    assert sr == 24000 and len(wa) == 1
    np.testing.assert_array_equal(wa[0], wb[0])
    # the reference demo's voice file ({"items": [asdict(item)]}, torch.save / torch.load(weights_only=True))
    import tempfile
    from qwen_tts import load_voice_clone_prompt, save_voice_clone_prompt
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "voice.pt")
        save_voice_clone_prompt(items, path)
        raw = torch.load(path, map_location="cpu", weights_only=True)
        assert set(raw["items"][0]) == {"ref_code", "ref_spk_embedding", "x_vector_only_mode", "icl_mode", "ref_text"}
        loaded = load_voice_clone_prompt(path)
    assert loaded[0].ref_text == "a reference transcript" and loaded[0].icl_mode
    wl, _ = tts.generate_voice_clone("hello there", language="English", voice_clone_prompt=loaded, **kw)
    np.testing.assert_array_equal(wa[0], wl[0])
    xv = tts.create_voice_clone_prompt((w, 24000), x_vector_only_mode=True)
    assert xv[0].ref_code is None and xv[0].x_vector_only_mode
    wc, _ = tts.generate_voice_clone("hello there", language="English", voice_clone_prompt=xv, **kw)
    assert wc[0].ndim == 1
    with pytest.raises(ValueError):
        tts.create_voice_clone_prompt((w, 24000))  # ICL mode needs ref_text


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_speaker_encoder_batched_clips_match_single(dtype):
    """embed_many: equal-length clips share one ECAPA pass (rows of one batch), other lengths get their own; every
    x-vector matches the clip's own embed()."""
    from cases import ref_audio
    se = _speaker("tiny-base", dtype)
    wavs = [ref_audio(24000, 10), ref_audio(24000, 11), ref_audio(30000, 12), ref_audio(24000, 13)]
    many = se.embed_many(wavs).cpu().numpy()
    for i, w in enumerate(wavs):
        one = se.embed(w).cpu().numpy()
        rel = np.linalg.norm(many[i] - one) / np.linalg.norm(one)
        assert rel < (1e-5 if dtype == "fp32" else 2e-2), (i, rel)
