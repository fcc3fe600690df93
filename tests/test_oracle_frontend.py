"""Pin the voice-clone front-end oracle (oracle/encoder.py, oracle/speaker.py) to the reference's own outputs.

Golden vectors: tests/golden/frontend_{tiny,full}.npz, written by tests/golden/make_golden.py (--only frontend),
which runs the reference `Qwen3TTSTokenizerV2Model.encode` (transformers MimiModel inside) and
`mel_spectrogram` + `Qwen3TTSSpeakerEncoder` via `extract_speaker_embedding` on seeded synthetic weights.
The slaney mel filterbank (librosa, absent offline) is the oracle's restatement on both sides of those fixtures; the
filterbank itself is pinned separately against the two librosa.filters.mel outputs the reference ships as data
(tests/golden/librosa_mel_filters.npz, tests/golden/copy_librosa_mel.py).  CPU only.
"""
import json
import os

import numpy as np
import pytest

from cases import frontend_cases, ref_audio
from oracle import load_preset, synth_param
from oracle.encoder import EncoderOracle, encoder_param_specs
from oracle.speaker import SpeakerOracle, mel_spectrogram, slaney_mel_filterbank, speaker_param_specs

GOLD = os.path.join(os.path.dirname(__file__), "golden")
CASES = [("tiny-base", "tiny", "frontend_tiny.npz"), ("1.7b-base", "full", "frontend_full.npz")]


def test_frontend_param_specs_match_reference():
    specs = json.load(open(os.path.join(GOLD, "param_specs.json")))
    for p in ("tiny-base", "1.7b-base", "0.6b-base", "1.7b-customvoice"):
        cfg, ccfg = load_preset(p)
        assert {k: list(v) for k, v in encoder_param_specs(ccfg)} == specs[p + "/encoder"]
        if p.endswith("base"):
            ref = {k: v for k, v in specs[p].items() if k.startswith("speaker_encoder.")}
            assert {k: list(v) for k, v in speaker_param_specs(cfg)} == ref


def test_slaney_filterbank_properties():
    """Structural checks of the restated filterbank (librosa itself is absent): triangles over [fmin, fmax],
    non-negative, slaney area normalisation (each band integrates to ~1 / bandwidth-scaled), empty above fmax."""
    w = slaney_mel_filterbank(24000, 1024, 128, 0, 12000)
    assert w.shape == (128, 513) and w.dtype == np.float32
    assert (w >= 0).all() and (w.sum(1) > 0).all()
    peaks = w.argmax(1)
    assert (np.diff(peaks) >= 0).all()  # band centres increase
    nz = [np.nonzero(r)[0] for r in w]
    assert all(len(z) and z[-1] - z[0] + 1 == len(z) for z in nz)  # one contiguous triangle per band


@pytest.mark.parametrize("n_mels", [80, 128])
def test_slaney_filterbank_matches_librosa_output(n_mels):
    """Oracle and product filterbanks == librosa.filters.mel(sr=16000, n_fft=400, n_mels) as the reference stores it
    (qwen_tts/core/tokenizer_25hz/vq/assets/mel_filters.npz; generating call at whisper_encoder.py:47-53): bit-exact
    float32."""
    from qwen_tts.speaker import mel_filterbank
    ref = np.load(os.path.join(GOLD, "librosa_mel_filters.npz"))[f"mel_{n_mels}"]
    np.testing.assert_array_equal(slaney_mel_filterbank(16000, 400, n_mels), ref)
    np.testing.assert_array_equal(mel_filterbank(16000, 400, n_mels, 0.0, 8000.0), ref)


@pytest.mark.parametrize("preset,kind,fname", CASES)
def test_encoder_oracle_matches_reference(preset, kind, fname):
    z = np.load(os.path.join(GOLD, fname))
    _, ccfg = load_preset(preset)
    eo = EncoderOracle(ccfg, {n: synth_param(n, s) for n, s in encoder_param_specs(ccfg)})
    for key, lens in frontend_cases()[kind]["enc"].items():
        wavs = [ref_audio(n, 1000 + 10 * i + n % 97) for i, n in enumerate(lens)]
        for j, w in enumerate(wavs):
            assert abs(float(w.astype(np.float64).sum()) - float(z[f"enc/{key}/sum{j}"])) < 1e-9
        for j, c in enumerate(eo.encode(wavs)):
            g = z[f"enc/{key}/codes{j}"]
            assert c.shape == g.shape == (-(-lens[j] // 1920), 16)
            np.testing.assert_array_equal(c.numpy(), g, err_msg=f"{preset}/{key}/{j}")


@pytest.mark.parametrize("preset,kind,fname", CASES)
def test_speaker_oracle_matches_reference(preset, kind, fname):
    import torch
    z = np.load(os.path.join(GOLD, fname))
    cfg, _ = load_preset(preset)
    so = SpeakerOracle(cfg, {n: synth_param(n, s) for n, s in speaker_param_specs(cfg)})
    for j, n in enumerate(frontend_cases()[kind]["spk"]):
        w = ref_audio(n, 2000 + j)
        mel = mel_spectrogram(torch.from_numpy(w)[None]).transpose(1, 2)[0].numpy()
        np.testing.assert_allclose(mel, z[f"spk/{j}/mel"], atol=1e-5, rtol=0)
        np.testing.assert_allclose(so.embed(w).numpy(), z[f"spk/{j}/emb"], atol=1e-4, rtol=1e-5)
