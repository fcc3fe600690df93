"""Drop-in `Qwen3TTSTokenizer` (reference: qwen_tts/inference/qwen3_tts_tokenizer.py, `Z` below).

decode() accepts exactly the reference's input forms (Z:286-329: encode output / dict / list of dicts,
torch or numpy codes, [T,16] or [B,T,16]), right-pads a batch with code 0 (Z:329) and returns
(list of 1-D float32 numpy wavs, 24000).  The decoder runs on the MI355X HIP kernels (qwen_tts/codec.py).
encode() (Z:208-257) takes the reference's audio forms, right-pads the batch like its
EncodecFeatureExtractor and runs the 12 Hz encoder on the HIP kernels (qwen_tts/encoder.py), returning an
object with `.audio_codes` = list of int64 [T_i, 16] device tensors (Qwen3TTSTokenizerV2EncoderOutput).
"""
from __future__ import annotations

import os
from typing import List, Optional, Tuple

import numpy as np
import torch
from torch.nn.utils.rnn import pad_sequence

from .. import audio as _audio
from ..codec import CodecDecoder
from ..encoder import TokenizerEncoder, encoder_specs
from ..weights import codec_specs, is_preset_dir, load_safetensors, read_json, resolve_path, synthetic


class EncoderOutput(dict):
    """Qwen3TTSTokenizerV2EncoderOutput (K:54-60): attribute and key access to `audio_codes`."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def to_tuple(self):
        return (self["audio_codes"],)


def _dtype_name(dtype) -> str:
    if dtype in (None, torch.bfloat16, "bf16", "bfloat16"):
        return "bf16"
    if dtype in (torch.float32, "fp32", "float32"):
        return "fp32"
    raise ValueError(f"unsupported dtype {dtype}")


class Qwen3TTSTokenizer:
    def __init__(self):
        self.model = None
        self.feature_extractor = None
        self.config = None
        self.device = None
        self.encoder = None

    @classmethod
    def from_pretrained(cls, pretrained_model_name_or_path: str, device_map="cuda:0", dtype=None, weights=None,
                        seed: int = 1234, **kwargs) -> "Qwen3TTSTokenizer":
        """Z:63-99.  `weights` (state dict keyed by reference names) overrides the files."""
        inst = cls()
        d = resolve_path(pretrained_model_name_or_path)
        if os.path.isdir(os.path.join(d, "speech_tokenizer")) and not os.path.exists(os.path.join(d, "config.json")):
            d = os.path.join(d, "speech_tokenizer")
        ccfg = read_json(os.path.join(d, "config.json"))
        if ccfg.get("model_type") != "qwen3_tts_tokenizer_12hz":
            raise ValueError(f"Unknown model type: {ccfg.get('model_type')} (only the 12 Hz tokenizer is on this path)")
        dev = torch.device(device_map if isinstance(device_map, str) and device_map.startswith("cuda") else "cuda:0")
        W = weights if weights is not None else load_safetensors(d)
        if not W:
            if not is_preset_dir(d):
                raise FileNotFoundError(f"no model*.safetensors in tokenizer directory {d!r}")
            W = synthetic(codec_specs(ccfg) + encoder_specs(ccfg), dev, seed)
        inst.config = ccfg
        inst.device = dev
        pre = os.path.join(d, "preprocessor_config.json")
        inst.feature_extractor = read_json(pre) if os.path.exists(pre) else {"sampling_rate": 24000}
        with torch.cuda.device(dev):
            inst.model = CodecDecoder(ccfg, W, dtype=_dtype_name(dtype), device=dev)
            if "encoder.encoder.layers.0.conv.weight" in W:
                inst.encoder = TokenizerEncoder(ccfg, W, dtype=_dtype_name(dtype), device=dev)
        return inst

    def encode(self, audios, sr: Optional[int] = None, return_dict: bool = True):
        """Z:208-257: wav path / base64 / np.ndarray (with sr) or lists of them -> EncoderOutput(audio_codes=[...])
        with int64 [T_i, 16] codes on the device (T_i = ceil(len_i / 1920) at 24 kHz)."""
        if self.encoder is None:
            raise ValueError("this tokenizer checkpoint has no encoder weights (encoder.* in model.safetensors)")
        target = int(self.feature_extractor.get("sampling_rate", 24000))
        wavs = _audio.normalize_at(audios, sr, target)
        with torch.inference_mode(), torch.cuda.device(self.device):
            codes = self.encoder.encode([torch.from_numpy(np.ascontiguousarray(w)) for w in wavs])
        if not return_dict:
            return (codes,)
        return EncoderOutput(audio_codes=codes)

    def decode(self, encoded) -> Tuple[List[np.ndarray], int]:
        """Z:259-365."""
        if hasattr(encoded, "audio_codes"):
            codes_list = encoded.audio_codes
        elif isinstance(encoded, dict):
            codes_list = encoded["audio_codes"]
        elif isinstance(encoded, list):
            codes_list = [e["audio_codes"] for e in encoded]
        else:
            raise TypeError("`encoded` must be an encode output, a dict, or a list of dicts.")
        if isinstance(codes_list, torch.Tensor):
            t = codes_list
            if t.dim() == 2:
                t = t.unsqueeze(0)
            padded = t.to(self.device)
        else:
            codes_list = [c if isinstance(c, torch.Tensor) else torch.from_numpy(np.asarray(c)).to(torch.long)
                          for c in codes_list]
            padded = pad_sequence(codes_list, batch_first=True, padding_value=0).to(self.device)
        with torch.inference_mode(), torch.cuda.device(self.device):
            wavs = self.model.decode(padded.long())
        return [w.to(torch.float32).cpu().numpy() for w in wavs], self.get_output_sample_rate()

    def get_model_type(self) -> str:
        return self.config["model_type"]

    def get_input_sample_rate(self) -> int:
        return int(self.config.get("input_sample_rate", 24000))

    def get_output_sample_rate(self) -> int:
        return int(self.config.get("output_sample_rate", 24000))

    def get_encode_downsample_rate(self) -> int:
        return int(self.config.get("encode_downsample_rate", 1920))

    def get_decode_upsample_rate(self) -> int:
        return int(self.config.get("decode_upsample_rate", 1920))
