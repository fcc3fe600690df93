"""Host-side reference-audio handling (qwen_tts/audio.py): the input forms of the reference wrappers
(W = qwen_tts/inference/qwen3_tts_model.py:188-264, Z = qwen_tts/inference/qwen3_tts_tokenizer.py:100-206) and the
resampler that stands in for librosa.resample (soxr; absent offline, so resampled inputs stay parity unpinned --
these tests pin its band-limited behaviour and librosa's output length, not soxr's bits).  CPU only."""
import base64
import struct

import numpy as np
import pytest

from qwen_tts import audio as A


def _wav(samples, sr, bits=16, ch=1, tag=1, extensible=False):
    """RIFF/WAVE bytes for int/float sample arrays ([n] or [n, ch], already in the target integer / float range)."""
    x = np.asarray(samples)
    if tag == 3:
        payload = x.astype("<f4" if bits == 32 else "<f8").tobytes()
    elif bits == 8:
        payload = x.astype(np.uint8).tobytes()
    elif bits == 16:
        payload = x.astype("<i2").tobytes()
    elif bits == 24:
        v = x.astype(np.int64).reshape(-1) & 0xFFFFFF
        payload = np.stack([v & 0xFF, (v >> 8) & 0xFF, (v >> 16) & 0xFF], 1).astype(np.uint8).tobytes()
    else:
        payload = x.astype("<i4").tobytes()
    ba = bits // 8 * ch
    fmt = struct.pack("<HHIIHH", 0xFFFE if extensible else tag, ch, sr, sr * ba, ba, bits)
    if extensible:
        fmt += struct.pack("<HHI", 22, bits, 0) + struct.pack("<H", tag) + b"\x00" * 14
    chunks = b"fmt " + struct.pack("<I", len(fmt)) + fmt
    chunks += b"LIST" + struct.pack("<I", 3) + b"abc\x00"  # odd-sized chunk: pad byte skipped
    chunks += b"data" + struct.pack("<I", len(payload)) + payload
    return b"RIFF" + struct.pack("<I", 4 + len(chunks)) + b"WAVE" + chunks


@pytest.mark.parametrize("bits,scale,tag", [(16, 32768.0, 1), (24, float(1 << 23), 1), (32, 2147483648.0, 1),
                                            (32, 1.0, 3), (64, 1.0, 3)])
def test_wav_pcm_and_float_decode(bits, scale, tag):
    rng = np.random.default_rng(bits + tag)
    if tag == 3:
        x = rng.uniform(-1, 1, 300)
        want = x.astype(np.float32)
    else:
        hi = int(scale) - 1
        x = rng.integers(-hi - 1, hi, 300)
        want = (x / scale).astype(np.float32)
    y, sr = A.read_wav_bytes(_wav(x, 16000, bits=bits, tag=tag))
    assert sr == 16000 and y.dtype == np.float32
    np.testing.assert_allclose(y, want, rtol=0, atol=1e-7)


def test_wav_8bit_stereo_extensible_and_mono_average(tmp_path):
    x = np.array([[0, 255], [128, 128], [64, 192]], dtype=np.uint8)
    data = _wav(x, 22050, bits=8, ch=2, extensible=True)
    y, sr = A.read_wav_bytes(data)
    assert sr == 22050 and y.shape == (3, 2)
    np.testing.assert_allclose(y, (x.astype(np.float32) - 128) / 128)
    p = tmp_path / "a.wav"
    p.write_bytes(data)
    m, sr2 = A.load_audio(str(p))  # W:207-223: channels averaged to mono
    assert sr2 == 22050
    np.testing.assert_allclose(m, y.mean(-1))


def test_base64_forms_and_detection():
    data = _wav(np.arange(-200, 200, 3), 24000)
    raw = base64.b64encode(data).decode()
    url = "data:audio/wav;base64," + raw
    # W:188-194's heuristic, quirks included: a raw string counts as base64 only without path separators
    assert A.is_probably_base64(url) and not A.is_probably_base64("/tmp/x.wav")
    assert A.is_probably_base64(raw) == ("/" not in raw and len(raw) > 256)
    assert A.is_probably_base64("A" * 257) and not A.is_probably_base64("A" * 256)
    a, _ = A.load_audio(url)
    np.testing.assert_array_equal(a, A.read_wav_bytes(A.decode_base64(raw))[0])
    assert A.is_url("https://x/y.wav") and not A.is_url("x.wav")


def test_bad_containers_raise():
    with pytest.raises(ValueError):
        A.read_wav_bytes(b"OggS" + b"\x00" * 40)
    with pytest.raises(ValueError):
        A.read_wav_bytes(b"RIFF" + struct.pack("<I", 4) + b"WAVE")


def test_resample_passthrough_and_length():
    y = np.random.default_rng(0).standard_normal(24001).astype(np.float32)
    np.testing.assert_array_equal(A.resample(y, 24000, 24000), y)  # the models' rate: untouched, as the reference
    for o, t, n in [(16000, 24000, 16001), (44100, 24000, 44101), (48000, 24000, 4801), (22050, 16000, 999)]:
        # librosa.resample(fix=True) returns ceil(n * t / o) samples
        assert A.resample(np.zeros(n, np.float32), o, t).shape[0] == int(np.ceil(n * t / o))


def test_resample_is_band_limited():
    """A tone below both Nyquists survives 16k -> 24k and 48k -> 24k (interior samples match the analytic tone);
    a tone above the target Nyquist is suppressed (anti-aliasing)."""
    for o in (16000, 48000):
        n = o  # 1 s
        t_in = np.arange(n) / o
        y = A.resample(np.sin(2 * np.pi * 440.0 * t_in).astype(np.float32), o, 24000)
        t_out = np.arange(y.shape[0]) / 24000
        ref = np.sin(2 * np.pi * 440.0 * t_out)
        mid = slice(2400, y.shape[0] - 2400)
        assert np.abs(y[mid] - ref[mid]).max() < 2e-3
    t_in = np.arange(48000) / 48000
    y = A.resample(np.sin(2 * np.pi * 15000.0 * t_in).astype(np.float32), 48000, 24000)
    assert np.sqrt(np.mean(y[2400:-2400] ** 2)) < 1e-2


def test_normalize_at_forms():
    y = np.ones((480, 2), np.float32)
    out = A.normalize_at([y], 48000, 24000)
    assert len(out) == 1 and out[0].ndim == 1 and out[0].shape[0] == 240
    with pytest.raises(ValueError):
        A.normalize_at([np.zeros(10, np.float32)], None, 24000)
    with pytest.raises(ValueError):
        A.normalize_pairs(np.zeros(10, np.float32))
    assert A.normalize_at([], None, 24000) == []
