"""Reference-audio input handling for the voice-clone front end (host side, before any kernel runs).

Mirrors the input forms of the reference wrappers (W = qwen_tts/inference/qwen3_tts_model.py:188-264,
Z = qwen_tts/inference/qwen3_tts_tokenizer.py:100-206): a wav path, an http(s) URL, a base64 string (raw or
`data:` URL), a (np.ndarray, sr) tuple or raw arrays with an explicit sr; multi-channel audio is averaged to
mono.  The reference decodes files with soundfile / librosa and resamples with `librosa.resample` (soxr);
neither library exists in this image, so:
  * files: RIFF/WAVE is parsed here (PCM 8/16/24/32-bit and IEEE float 32/64); other containers raise.
  * resampling: scipy.signal.resample_poly (Kaiser-windowed polyphase FIR).  Its output is not bit-identical to
    soxr's, so inputs that need resampling are "parity unpinned"; 24 kHz input (the models' rate) is passed
    through untouched, exactly like the reference.
"""
from __future__ import annotations

import base64
import io
import struct
import urllib.request
from fractions import Fraction
from typing import List, Tuple

import numpy as np


def is_url(s: str) -> bool:
    return s.startswith("http://") or s.startswith("https://")


def is_probably_base64(s: str) -> bool:
    """W:188-194."""
    if s.startswith("data:audio"):
        return True
    if ("/" not in s and "\\" not in s) and len(s) > 256:
        return True
    return False


def decode_base64(b64: str) -> bytes:
    if "," in b64 and b64.strip().startswith("data:"):
        b64 = b64.split(",", 1)[1]
    return base64.b64decode(b64)


def read_wav_bytes(data: bytes) -> Tuple[np.ndarray, int]:
    """RIFF/WAVE -> (float32 [n] or [n, ch], sr)."""
    f = io.BytesIO(data)
    riff = f.read(12)
    if len(riff) < 12 or riff[:4] != b"RIFF" or riff[8:12] != b"WAVE":
        raise ValueError("unsupported audio container (only RIFF/WAVE can be decoded without soundfile/librosa)")
    fmt, payload = None, None
    while True:
        hdr = f.read(8)
        if len(hdr) < 8:
            break
        cid, size = hdr[:4], struct.unpack("<I", hdr[4:])[0]
        body = f.read(size)
        if size % 2:
            f.read(1)
        if cid == b"fmt ":
            fmt = body
        elif cid == b"data":
            payload = body
    if fmt is None or payload is None:
        raise ValueError("malformed WAVE file (missing fmt or data chunk)")
    tag, ch, sr, _, _, bits = struct.unpack("<HHIIHH", fmt[:16])
    if tag == 0xFFFE and len(fmt) >= 26:  # WAVE_FORMAT_EXTENSIBLE: the subformat's first 2 bytes are the tag
        tag = struct.unpack("<H", fmt[24:26])[0]
    if tag == 1:
        if bits == 8:
            x = (np.frombuffer(payload, np.uint8).astype(np.float32) - 128.0) / 128.0
        elif bits == 16:
            x = np.frombuffer(payload, "<i2").astype(np.float32) / 32768.0
        elif bits == 24:
            b = np.frombuffer(payload[: len(payload) // 3 * 3], np.uint8).reshape(-1, 3).astype(np.int32)
            v = b[:, 0] | (b[:, 1] << 8) | (b[:, 2] << 16)
            v = np.where(v >= 1 << 23, v - (1 << 24), v)
            x = v.astype(np.float32) / float(1 << 23)
        elif bits == 32:
            x = np.frombuffer(payload, "<i4").astype(np.float32) / 2147483648.0
        else:
            raise ValueError(f"unsupported PCM bit depth {bits}")
    elif tag == 3:
        x = np.frombuffer(payload, "<f4" if bits == 32 else "<f8").astype(np.float32)
    else:
        raise ValueError(f"unsupported WAVE format tag {tag}")
    n = len(x) // ch * ch
    x = x[:n]
    return (x.reshape(-1, ch) if ch > 1 else x), int(sr)


def load_audio(x: str) -> Tuple[np.ndarray, int]:
    """W:207-223: path / URL / base64 -> (mono float32, sr)."""
    if is_url(x):
        with urllib.request.urlopen(x) as resp:
            data = resp.read()
    elif is_probably_base64(x):
        data = decode_base64(x)
    else:
        with open(x, "rb") as fh:
            data = fh.read()
    audio, sr = read_wav_bytes(data)
    if audio.ndim > 1:
        audio = np.mean(audio, axis=-1)
    return audio.astype(np.float32), int(sr)


def resample(y: np.ndarray, orig_sr: int, target_sr: int) -> np.ndarray:
    """Band-limited rational resampling (stands in for librosa.resample; parity unpinned, see module doc)."""
    if int(orig_sr) == int(target_sr):
        return y.astype(np.float32)
    from scipy.signal import resample_poly
    fr = Fraction(int(target_sr), int(orig_sr))
    return resample_poly(y.astype(np.float64), fr.numerator, fr.denominator).astype(np.float32)


def normalize_pairs(audios) -> List[Tuple[np.ndarray, int]]:
    """W:225-264: list of (mono float32 wav, original sr)."""
    items = audios if isinstance(audios, list) else [audios]
    out = []
    for a in items:
        if isinstance(a, str):
            out.append(load_audio(a))
        elif isinstance(a, tuple) and len(a) == 2 and isinstance(a[0], np.ndarray):
            out.append((a[0].astype(np.float32), int(a[1])))
        elif isinstance(a, np.ndarray):
            raise ValueError("For numpy waveform input, pass a tuple (audio, sr).")
        else:
            raise TypeError(f"Unsupported audio input type: {type(a)}")
    return [((w if w.ndim == 1 else np.mean(w, axis=-1)).astype(np.float32), sr) for w, sr in out]


def normalize_at(audios, sr, target_sr: int) -> List[np.ndarray]:
    """Z:160-206: list of mono float32 waveforms at target_sr."""
    if isinstance(audios, (str, np.ndarray)):
        audios = [audios]
    if len(audios) == 0:
        return []
    if isinstance(audios[0], str):
        out = []
        for x in audios:
            a, s = load_audio(x)
            out.append(resample(a, s, target_sr))
        return out
    if sr is None:
        raise ValueError("For numpy waveform input, you must provide `sr` (original sampling rate).")
    out = []
    for a in audios:
        if not isinstance(a, np.ndarray):
            raise TypeError("Mixed input types are not supported. Use all paths/base64 or all numpy arrays.")
        if a.ndim > 1:
            a = np.mean(a, axis=-1)
        out.append(resample(a.astype(np.float32), int(sr), target_sr))
    return out
