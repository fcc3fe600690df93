"""Drop-in `Qwen3TTSModel` (reference: qwen_tts/inference/qwen3_tts_model.py, `W` below).

Same public surface and semantics: from_pretrained, generate_custom_voice / generate_voice_design /
generate_voice_clone (from reference audio or a prepared voice_clone_prompt), create_voice_clone_prompt,
get_supported_speakers / languages, kwargs
precedence of `_merge_generate_kwargs` (W:287-352), validation errors (W:141-186), wrapper defaults
(max_new_tokens 2048, non_streaming_mode True/True/False) and the 0.6B instruct drop (W:799).
New: `stream()` yields (pcm chunk, sr) per utterance as soon as its codes are decoded.
All compute runs on the MI355X engine (qwen_tts/model.py + qwen_tts/codec.py).
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Any, Dict, List, Optional, Tuple, Union

import numpy as np
import torch

from .. import audio as _audio
from .. import kernels as _kernels
from ..model import TTSModel
from ..text import load_processor
from ..speaker import speaker_specs
from ..weights import is_preset_dir, load_safetensors, read_json, resolve_path, synthetic, talker_specs
from .qwen3_tts_tokenizer import Qwen3TTSTokenizer, _dtype_name

AudioLike = Union[str, np.ndarray, Tuple[np.ndarray, int]]
MaybeList = Union[Any, List[Any]]


@dataclass
class VoiceClonePromptItem:
    """W:40-51."""
    ref_code: Optional[torch.Tensor]
    ref_spk_embedding: torch.Tensor
    x_vector_only_mode: bool
    icl_mode: bool
    ref_text: Optional[str] = None


def save_voice_clone_prompt(items: List[VoiceClonePromptItem], path: str) -> None:
    """The reference demo's voice file (qwen_tts/cli/demo.py:514-521): torch.save({"items": [asdict(item)]}),
    tensors moved to the CPU so the file loads anywhere."""
    from dataclasses import asdict
    out = []
    for it in items:
        d = asdict(it)
        for k in ("ref_code", "ref_spk_embedding"):
            if isinstance(d[k], torch.Tensor):
                d[k] = d[k].detach().cpu()
        out.append(d)
    torch.save({"items": out}, path)


def load_voice_clone_prompt(path: str) -> List[VoiceClonePromptItem]:
    """Read a voice file written by save_voice_clone_prompt or the reference demo (demo.py:527-563), with
    torch.load(weights_only=True) like the reference: no code in the file is executed."""
    payload = torch.load(path, map_location="cpu", weights_only=True)
    if not isinstance(payload, dict) or "items" not in payload:
        raise ValueError("Invalid file format")
    raw = payload["items"]
    if not isinstance(raw, list) or len(raw) == 0:
        raise ValueError("Empty voice items")
    items = []
    for d in raw:
        if not isinstance(d, dict):
            raise ValueError("Invalid item format in file")
        ref_code = d.get("ref_code", None)
        if ref_code is not None and not torch.is_tensor(ref_code):
            ref_code = torch.tensor(ref_code)
        spk = d.get("ref_spk_embedding", None)
        if spk is None:
            raise ValueError("Missing ref_spk_embedding")
        if not torch.is_tensor(spk):
            spk = torch.tensor(spk)
        xv = bool(d.get("x_vector_only_mode", False))
        items.append(VoiceClonePromptItem(ref_code=ref_code, ref_spk_embedding=spk, x_vector_only_mode=xv,
                                          icl_mode=bool(d.get("icl_mode", not xv)), ref_text=d.get("ref_text", None)))
    return items


class Qwen3TTSModel:
    def __init__(self, model: TTSModel, processor, generate_defaults: Optional[Dict[str, Any]] = None):
        self.model = model
        self.processor = processor
        self.generate_defaults = generate_defaults or {}
        self.device = model.device

    @classmethod
    def from_pretrained(cls, pretrained_model_name_or_path: str, device_map="cuda:0", dtype=None,
                        attn_implementation=None, weights=None, codec_weights=None, seed: int = 1234,
                        **kwargs) -> "Qwen3TTSModel":
        """W:82-121.  A local checkpoint dir (config.json, generation_config.json, model*.safetensors,
        speech_tokenizer/) or a synthetic preset / hub id (offline: synthetic weights).  `attn_implementation`
        is accepted for API compatibility; attention always runs on the HIP kernel."""
        d = resolve_path(pretrained_model_name_or_path)
        cfg = read_json(os.path.join(d, "config.json"))
        if cfg.get("model_type") != "qwen3_tts":
            raise TypeError(f"expected a qwen3_tts checkpoint, got model_type={cfg.get('model_type')!r}")
        gpath = os.path.join(d, "generation_config.json")
        gen = read_json(gpath) if os.path.exists(gpath) else {}
        dev = torch.device(device_map if isinstance(device_map, str) and device_map.startswith("cuda") else "cuda:0")
        W = weights if weights is not None else load_safetensors(d)
        if not W:
            if not is_preset_dir(d):
                raise FileNotFoundError(f"no model*.safetensors in checkpoint directory {d!r}")
            specs = talker_specs(cfg)
            if cfg.get("tts_model_type") == "base":
                specs = specs + speaker_specs(cfg)
            W = synthetic(specs, dev, seed)
        with torch.cuda.device(dev):
            m = TTSModel(cfg, W, dtype=_dtype_name(dtype), device=dev, generate_config=gen)
        del W
        m.load_speech_tokenizer(Qwen3TTSTokenizer.from_pretrained(os.path.join(d, "speech_tokenizer"), device_map=dev,
                                                                  dtype=dtype, weights=codec_weights, seed=seed))
        return cls(m, load_processor(d), gen)

    # ---------------------------------------------------------------- validation (W:123-186)
    def _supported_languages_set(self):
        v = self.model.get_supported_languages()
        return None if v is None else set(str(x).lower() for x in v)

    def _supported_speakers_set(self):
        v = self.model.get_supported_speakers()
        return None if v is None else set(str(x).lower() for x in v)

    def _validate_languages(self, languages):
        sup = self._supported_languages_set()
        if sup is None:
            return
        bad = [x for x in languages if x is None or str(x).lower() not in sup]
        if bad:
            raise ValueError(f"Unsupported languages: {bad}. Supported: {sorted(sup)}")

    def _validate_speakers(self, speakers):
        sup = self._supported_speakers_set()
        if sup is None:
            return
        bad = [s for s in speakers if s not in (None, "") and str(s).lower() not in sup]
        if bad:
            raise ValueError(f"Unsupported speakers: {bad}. Supported: {sorted(sup)}")

    def _ensure_list(self, x: MaybeList) -> List[Any]:
        return x if isinstance(x, list) else [x]

    def _build_assistant_text(self, text: str) -> str:
        return f"<|im_start|>assistant\n{text}<|im_end|>\n<|im_start|>assistant\n"

    def _build_ref_text(self, text: str) -> str:
        return f"<|im_start|>assistant\n{text}<|im_end|>\n"

    def _build_instruct_text(self, instruct: str) -> str:
        return f"<|im_start|>user\n{instruct}<|im_end|>\n"

    def _tokenize_texts(self, texts: List[str]) -> List[torch.Tensor]:
        out = []
        for t in texts:
            ids = self.processor(text=t, return_tensors="pt", padding=True)["input_ids"]
            out.append(ids.unsqueeze(0) if ids.dim() == 1 else ids)
        return out

    def _merge_generate_kwargs(self, do_sample=None, top_k=None, top_p=None, temperature=None, repetition_penalty=None,
                               subtalker_dosample=None, subtalker_top_k=None, subtalker_top_p=None,
                               subtalker_temperature=None, max_new_tokens=None, **kwargs) -> Dict[str, Any]:
        """W:287-352: user value > generation_config.json > hard default."""
        hard = dict(do_sample=True, top_k=50, top_p=1.0, temperature=0.9, repetition_penalty=1.05,
                    subtalker_dosample=True, subtalker_top_k=50, subtalker_top_p=1.0, subtalker_temperature=0.9,
                    max_new_tokens=2048)

        def pick(name, v):
            if v is not None:
                return v
            if name in self.generate_defaults:
                return self.generate_defaults[name]
            return hard[name]

        merged = dict(kwargs)
        merged.update(do_sample=pick("do_sample", do_sample), top_k=pick("top_k", top_k), top_p=pick("top_p", top_p),
                      temperature=pick("temperature", temperature),
                      repetition_penalty=pick("repetition_penalty", repetition_penalty),
                      subtalker_dosample=pick("subtalker_dosample", subtalker_dosample),
                      subtalker_top_k=pick("subtalker_top_k", subtalker_top_k),
                      subtalker_top_p=pick("subtalker_top_p", subtalker_top_p),
                      subtalker_temperature=pick("subtalker_temperature", subtalker_temperature),
                      max_new_tokens=pick("max_new_tokens", max_new_tokens))
        return merged

    def _decode(self, codes_list):
        return self.model.speech_tokenizer.decode([{"audio_codes": c} for c in codes_list])

    # ---------------------------------------------------------------- voice clone (W:356-633)
    def create_voice_clone_prompt(self, ref_audio, ref_text=None, x_vector_only_mode=False) -> List[VoiceClonePromptItem]:
        """W:356-458: reference audio -> ref_code (12 Hz tokenizer encode, HIP) + x-vector (mel + ECAPA, HIP)."""
        if self.model.tts_model_type != "base":
            raise ValueError(f"model with \ntokenizer_type: {self.model.tokenizer_type}\n"
                             f"tts_model_size: {self.model.tts_model_size}\n"
                             f"tts_model_type: {self.model.tts_model_type}\n"
                             "does not support create_voice_clone_prompt, Please check Model Card or Readme for more details.")
        ref_audio_list = self._ensure_list(ref_audio)
        ref_text_list = self._ensure_list(ref_text) if isinstance(ref_text, list) else [ref_text] * len(ref_audio_list)
        xvec_list = self._ensure_list(x_vector_only_mode) if isinstance(x_vector_only_mode, list) else \
            [x_vector_only_mode] * len(ref_audio_list)
        if len(ref_text_list) != len(ref_audio_list) or len(xvec_list) != len(ref_audio_list):
            raise ValueError(f"Batch size mismatch: ref_audio={len(ref_audio_list)}, ref_text={len(ref_text_list)}, "
                             f"x_vector_only_mode={len(xvec_list)}")
        normalized = _audio.normalize_pairs(ref_audio_list)
        srs = [sr for _, sr in normalized]
        tok = self.model.speech_tokenizer
        spk_sr = self.model.speaker_encoder_sample_rate
        for i, (rtext, xvec_only) in enumerate(zip(ref_text_list, xvec_list)):
            if not xvec_only and (rtext is None or rtext == ""):
                raise ValueError(f"ref_text is required when x_vector_only_mode=False (ICL mode). Bad index={i}")
        # x-vectors of all clips (W:434 per clip; equal-length clips share one ECAPA pass here) on a side stream with
        # its own split-K workspace, concurrently with the tokenizer encode on this one (the two front ends are
        # independent; ~1.2 and ~3 ms of GPU work for four 3 s clips).  The encode is issued first: its GPU time
        # outlasts its host launch time, so the x-vector launches that follow land beside queued encoder work.
        dev = torch.device(self.model.device)
        main = torch.cuda.current_stream(dev)
        side = _kernels.side_stream(dev)
        side.wait_stream(main)
        if len(set(srs)) == 1:
            ref_codes = tok.encode([w for w, _ in normalized], sr=srs[0]).audio_codes
        else:
            ref_codes = [tok.encode(w, sr=sr).audio_codes[0] for w, sr in normalized]
        if getattr(self, "_side_ws", None) is None:
            self._side_ws = _kernels.new_workspace(dev)
        with torch.cuda.stream(side), _kernels.use_workspace(self._side_ws):
            spks = self.model.extract_speaker_embeddings(
                [_audio.resample(wav, sr, spk_sr) if sr != spk_sr else wav for wav, sr in normalized], sr=spk_sr)
        main.wait_stream(side)
        spks.record_stream(main)
        items = []
        for i, ((wav, sr), code, rtext, xvec_only) in enumerate(zip(normalized, ref_codes, ref_text_list, xvec_list)):
            spk = spks[i]
            items.append(VoiceClonePromptItem(ref_code=None if xvec_only else code, ref_spk_embedding=spk,
                                              x_vector_only_mode=bool(xvec_only), icl_mode=bool(not xvec_only),
                                              ref_text=rtext))
        return items

    def _prompt_items_to_voice_clone_prompt(self, items: List[VoiceClonePromptItem]) -> Dict[str, Any]:
        return dict(ref_code=[it.ref_code for it in items], ref_spk_embedding=[it.ref_spk_embedding for it in items],
                    x_vector_only_mode=[it.x_vector_only_mode for it in items], icl_mode=[it.icl_mode for it in items])

    @torch.no_grad()
    def generate_voice_clone(self, text, language=None, ref_audio=None, ref_text=None, x_vector_only_mode=False,
                             voice_clone_prompt=None, non_streaming_mode=False, **kwargs):
        input_ids, ref_ids, vcp, languages = self._voice_clone_inputs(text, language, ref_audio, ref_text,
                                                                      x_vector_only_mode, voice_clone_prompt)
        codes, _ = self.model.generate(input_ids=input_ids, ref_ids=ref_ids, voice_clone_prompt=vcp, languages=languages,
                                       non_streaming_mode=non_streaming_mode, **self._merge_generate_kwargs(**kwargs))
        refs = vcp.get("ref_code", None)
        dec = [torch.cat([refs[i].cpu().long(), c], 0) if refs is not None and refs[i] is not None else c
               for i, c in enumerate(codes)]
        wavs, fs = self._decode(dec)
        out = []
        for i, w in enumerate(wavs):
            if refs is not None and refs[i] is not None:
                cut = int(int(refs[i].shape[0]) / max(int(dec[i].shape[0]), 1) * w.shape[0])
                out.append(w[cut:])
            else:
                out.append(w)
        return out, fs

    @torch.no_grad()
    def stream_voice_clone(self, text, language=None, ref_audio=None, ref_text=None, x_vector_only_mode=False,
                           voice_clone_prompt=None, non_streaming_mode=False, first_chunk_frames=1, chunk_frames=48,
                           **kwargs):
        """New surface (no reference counterpart, SURVEY.md §8f-1 + 8f-2): streaming voice clone.  Same inputs as
        generate_voice_clone (reference audio is encoded / x-vectored at submit); yields (utterance index, pcm chunk
        np.float32, sample rate, is_last).  Per utterance the chunks concatenate to generate_voice_clone()'s PCM: in
        ICL mode the reference codes are decoded in front of the generated ones and the output starts at their
        boundary -- the wrapper's proportional cut keeps floor(555 R / T) more samples of the reference's tail, a
        length-dependent point a stream cannot know in advance (TTSModel._stream_stateful)."""
        input_ids, ref_ids, vcp, languages = self._voice_clone_inputs(text, language, ref_audio, ref_text,
                                                                      x_vector_only_mode, voice_clone_prompt)
        sr = self.model.speech_tokenizer.get_output_sample_rate()
        for i, pcm, last in self.model.stream(input_ids=input_ids, ref_ids=ref_ids, voice_clone_prompt=vcp,
                                              languages=languages, non_streaming_mode=non_streaming_mode,
                                              first_chunk_frames=first_chunk_frames, chunk_frames=chunk_frames,
                                              **self._merge_generate_kwargs(**kwargs)):
            yield i, pcm.to(torch.float32).cpu().numpy(), sr, last

    def _voice_clone_inputs(self, text, language, ref_audio, ref_text, x_vector_only_mode, voice_clone_prompt):
        """W:460-633 input handling of generate_voice_clone: -> (input_ids, ref_ids, voice_clone_prompt dict,
        languages)."""
        if self.model.tts_model_type != "base":
            raise ValueError(f"model with tts_model_type: {self.model.tts_model_type} does not support "
                             "generate_voice_clone, Please check Model Card or Readme for more details.")
        texts = self._ensure_list(text)
        languages = self._ensure_list(language) if isinstance(language, list) else \
            ([language] * len(texts) if language is not None else ["Auto"] * len(texts))
        if len(languages) == 1 and len(texts) > 1:
            languages = languages * len(texts)
        if len(texts) != len(languages):
            raise ValueError(f"Batch size mismatch: text={len(texts)}, language={len(languages)}")
        self._validate_languages(languages)
        if voice_clone_prompt is None:
            if ref_audio is None:
                raise ValueError("Either `voice_clone_prompt` or `ref_audio` must be provided.")
            items = self.create_voice_clone_prompt(ref_audio, ref_text, x_vector_only_mode)
            if len(items) == 1 and len(texts) > 1:  # one reference voice for a batch of texts (W:567-571)
                items = items * len(texts)
            if len(items) != len(texts):
                raise ValueError(f"Batch size mismatch: prompt={len(items)}, text={len(texts)}")
            vcp, ref_texts = self._prompt_items_to_voice_clone_prompt(items), [it.ref_text for it in items]
        elif isinstance(voice_clone_prompt, list):
            items = voice_clone_prompt
            if len(items) == 1 and len(texts) > 1:
                items = items * len(texts)
            if len(items) != len(texts):
                raise ValueError(f"Batch size mismatch: prompt={len(items)}, text={len(texts)}")
            vcp, ref_texts = self._prompt_items_to_voice_clone_prompt(items), [it.ref_text for it in items]
        else:
            vcp, ref_texts = voice_clone_prompt, None
        input_ids = self._tokenize_texts([self._build_assistant_text(t) for t in texts])
        ref_ids = None
        if ref_texts is not None:
            ref_ids = [None if not rt else self._tokenize_texts([self._build_ref_text(rt)])[0] for rt in ref_texts]
        return input_ids, ref_ids, vcp, languages

    # ---------------------------------------------------------------- voice design (W:637-728)
    @torch.no_grad()
    def generate_voice_design(self, text, instruct, language=None, non_streaming_mode=True, **kwargs):
        if self.model.tts_model_type != "voice_design":
            raise ValueError(f"model with tts_model_type: {self.model.tts_model_type} does not support "
                             "generate_voice_design, Please check Model Card or Readme for more details.")
        texts = self._ensure_list(text)
        languages = self._ensure_list(language) if isinstance(language, list) else \
            ([language] * len(texts) if language is not None else ["Auto"] * len(texts))
        instructs = self._ensure_list(instruct)
        if len(languages) == 1 and len(texts) > 1:
            languages = languages * len(texts)
        if len(instructs) == 1 and len(texts) > 1:
            instructs = instructs * len(texts)
        if not (len(texts) == len(languages) == len(instructs)):
            raise ValueError(f"Batch size mismatch: text={len(texts)}, language={len(languages)}, "
                             f"instruct={len(instructs)}")
        self._validate_languages(languages)
        input_ids = self._tokenize_texts([self._build_assistant_text(t) for t in texts])
        ins_ids = [None if not x else self._tokenize_texts([self._build_instruct_text(x)])[0] for x in instructs]
        codes, _ = self.model.generate(input_ids=input_ids, instruct_ids=ins_ids, languages=languages,
                                       non_streaming_mode=non_streaming_mode, **self._merge_generate_kwargs(**kwargs))
        return self._decode(codes)

    # ---------------------------------------------------------------- custom voice (W:732-839)
    def _custom_voice_inputs(self, text, speaker, language, instruct):
        if self.model.tts_model_type != "custom_voice":
            raise ValueError(f"model with tts_model_type: {self.model.tts_model_type} does not support "
                             "generate_custom_voice, Please check Model Card or Readme for more details.")
        texts = self._ensure_list(text)
        languages = self._ensure_list(language) if isinstance(language, list) else \
            ([language] * len(texts) if language is not None else ["Auto"] * len(texts))
        speakers = self._ensure_list(speaker)
        if self.model.tts_model_size in "0b6":  # W:799 (substring test, kept as-is)
            instruct = None
        instructs = self._ensure_list(instruct) if isinstance(instruct, list) else \
            ([instruct] * len(texts) if instruct is not None else [""] * len(texts))
        if len(languages) == 1 and len(texts) > 1:
            languages = languages * len(texts)
        if len(speakers) == 1 and len(texts) > 1:
            speakers = speakers * len(texts)
        if len(instructs) == 1 and len(texts) > 1:
            instructs = instructs * len(texts)
        if not (len(texts) == len(languages) == len(speakers) == len(instructs)):
            raise ValueError(f"Batch size mismatch: text={len(texts)}, language={len(languages)}, "
                             f"speaker={len(speakers)}, instruct={len(instructs)}")
        self._validate_languages(languages)
        self._validate_speakers(speakers)
        input_ids = self._tokenize_texts([self._build_assistant_text(t) for t in texts])
        ins_ids = [None if not x else self._tokenize_texts([self._build_instruct_text(x)])[0] for x in instructs]
        return input_ids, ins_ids, languages, speakers

    @torch.no_grad()
    def generate_custom_voice(self, text, speaker, language=None, instruct=None, non_streaming_mode=True, **kwargs):
        input_ids, ins_ids, languages, speakers = self._custom_voice_inputs(text, speaker, language, instruct)
        codes, _ = self.model.generate(input_ids=input_ids, instruct_ids=ins_ids, languages=languages,
                                       speakers=speakers, non_streaming_mode=non_streaming_mode,
                                       **self._merge_generate_kwargs(**kwargs))
        return self._decode(codes)

    @torch.no_grad()
    def stream(self, text, speaker=None, language=None, instruct=None, non_streaming_mode=True,
               first_chunk_frames=1, chunk_frames=48, left_context=None, **kwargs):
        """New surface (no reference counterpart): streaming custom-voice generation.
        Yields (utterance index, pcm chunk np.float32, sample rate, is_last) while the batch decodes: the first
        chunk arrives after prefill + `first_chunk_frames` decode frames (1 frame: 1365 samples = 57 ms of audio,
        which outlasts the ~9 ms the next 2-frame chunk takes), later chunks double in size up to `chunk_frames`
        (each chunk's audio outlasts the generation of the next).  Per utterance the
        chunks concatenate to the one-shot generate_custom_voice() length and equal its PCM up to fp summation order
        (a stateful incremental codec decode; codes are identical -- see TTSModel.stream for the chunk rule and the
        stateless `left_context` form)."""
        input_ids, ins_ids, languages, speakers = self._custom_voice_inputs(text, speaker, language, instruct)
        sr = self.model.speech_tokenizer.get_output_sample_rate()
        for i, pcm, last in self.model.stream(input_ids=input_ids, instruct_ids=ins_ids, languages=languages,
                                              speakers=speakers, non_streaming_mode=non_streaming_mode,
                                              first_chunk_frames=first_chunk_frames, chunk_frames=chunk_frames,
                                              left_context=left_context, **self._merge_generate_kwargs(**kwargs)):
            yield i, pcm.to(torch.float32).cpu().numpy(), sr, last

    def get_supported_speakers(self) -> Optional[List[str]]:
        s = self._supported_speakers_set()
        return None if s is None else sorted(s)

    def get_supported_languages(self) -> Optional[List[str]]:
        s = self._supported_languages_set()
        return None if s is None else sorted(s)
