"""Import the read-only reference (`/root/reference/qwen_tts`) in THIS container for fixture generation.

TEST INFRASTRUCTURE ONLY.  Used by `tests/golden/make_golden.py` to produce golden vectors from the
reference itself; nothing on the GPU box (tests -m gpu, smoke(), bench.py) imports this file, and
`/root/reference` does not exist there.

The reference pins transformers==4.57.3 (`pyproject.toml:24`); this image has transformers 5.15.
The process-local patches below bend the 5.x entry points the reference calls back
to the 4.57 semantics.  The reference files themselves are untouched and are imported from their
original location.
"""
from __future__ import annotations

import functools
import importlib.machinery
import sys
import types

import torch

REF_ROOT = "/root/reference"

_loaded = {}


def _stub_module(name, **attrs):
    m = types.ModuleType(name)
    m.__spec__ = importlib.machinery.ModuleSpec(name, None)
    for k, v in attrs.items():
        setattr(m, k, v)
    sys.modules[name] = m
    return m


def _default_rope_init(config, device=None, *args, **kwargs):
    """Patch 2: the 4.57 'default' rope init, inv_freq = 1 / theta^(2i/d), attention scaling 1."""
    base = getattr(config, "rope_theta", None)
    if base is None:
        base = config.rope_parameters["rope_theta"]
    dim = getattr(config, "head_dim", None) or config.hidden_size // config.num_attention_heads
    inv_freq = 1.0 / (base ** (torch.arange(0, dim, 2, dtype=torch.int64).to(device=device, dtype=torch.float) / dim))
    return inv_freq, 1.0


def _make_mask_fn(sliding: bool):
    """Patch 3: 4.57-style additive 4D eager mask.

    allowed(q, kv) = kv <= cache_position[q]  and  mask2d[b, kv]  (and kv > cache_position[q] - window).
    """

    def fn(config=None, input_embeds=None, attention_mask=None, cache_position=None, past_key_values=None,
           position_ids=None, inputs_embeds=None, **kw):
        emb = input_embeds if input_embeds is not None else inputs_embeds
        bsz, q_len = emb.shape[0], emb.shape[1]
        past = past_key_values.get_seq_length() if past_key_values is not None else 0
        kv_len = past + q_len
        if cache_position is None:
            cache_position = torch.arange(past, past + q_len, device=emb.device)
        kv_idx = torch.arange(kv_len, device=emb.device)
        allowed = kv_idx[None, :] <= cache_position[:, None]  # [Q, KV]
        if sliding:
            window = config.sliding_window
            allowed = allowed & (kv_idx[None, :] > cache_position[:, None] - window)
        allowed = allowed[None, None].expand(bsz, 1, q_len, kv_len)
        if attention_mask is not None and attention_mask.dim() == 2:
            allowed = allowed & attention_mask[:, None, None, :kv_len].bool()
        mask = torch.zeros(allowed.shape, dtype=emb.dtype, device=emb.device)
        mask.masked_fill_(~allowed, torch.finfo(emb.dtype).min)
        return mask

    return fn


def _inject_cache_position(forward):
    """Patch 6: 5.x generate no longer passes `cache_position`; recreate it as arange(past, past+q)."""

    @functools.wraps(forward)
    def wrapped(*args, **kwargs):
        if kwargs.get("cache_position") is None:
            pkv = kwargs.get("past_key_values")
            past = pkv.get_seq_length() if pkv is not None else 0
            if kwargs.get("inputs_embeds") is not None:
                q = kwargs["inputs_embeds"].shape[1]
                dev = kwargs["inputs_embeds"].device
            else:
                q = kwargs["input_ids"].shape[1]
                dev = kwargs["input_ids"].device
            kwargs["cache_position"] = torch.arange(past, past + q, device=dev)
        return forward(*args, **kwargs)

    return wrapped


def load_reference():
    """Return (modeling_qwen3_tts, configuration_qwen3_tts, modeling_tokenizer_v2, configuration_tokenizer_v2)."""
    if _loaded:
        return _loaded["mods"]
    # transformers audio/Mimi modules must be imported before librosa is stubbed (they probe for it).
    import transformers.audio_utils  # noqa: F401
    from transformers import MimiConfig, MimiModel  # noqa: F401
    import transformers.utils.generic as tgeneric
    import transformers.modeling_rope_utils as trope
    import transformers.masking_utils as tmask

    # Patch 1: the reference uses the 4.57 factory form `@check_model_inputs()`.
    def check_model_inputs(func=None, **kw):
        if func is None:
            return lambda f: f
        return func

    tgeneric.check_model_inputs = check_model_inputs
    # Patch 2
    trope.ROPE_INIT_FUNCTIONS["default"] = _default_rope_init
    # Patch 4: librosa / soundfile are not installed; mel is not on the hot path.
    def _mel(*a, **k):
        raise RuntimeError("librosa.filters.mel is stubbed (not on the hot path)")

    lib = _stub_module("librosa", load=None, resample=None)
    lib.filters = _stub_module("librosa.filters", mel=_mel)
    _stub_module("soundfile")
    # Patch 5: package stubs skip qwen_tts/__init__.py and the 25 Hz tokenizer.
    if REF_ROOT not in sys.path:
        sys.path.insert(0, REF_ROOT)
    pkg = _stub_module("qwen_tts")
    pkg.__path__ = [REF_ROOT + "/qwen_tts"]
    inf = _stub_module("qwen_tts.inference")
    inf.__path__ = [REF_ROOT + "/qwen_tts/inference"]
    core = _stub_module("qwen_tts.core")
    core.__path__ = [REF_ROOT + "/qwen_tts/core"]
    import importlib

    ctok = importlib.import_module("qwen_tts.core.tokenizer_12hz.configuration_qwen3_tts_tokenizer_v2")
    mtok = importlib.import_module("qwen_tts.core.tokenizer_12hz.modeling_qwen3_tts_tokenizer_v2")

    class _V1Stub:  # 25 Hz tokenizer needs sox/onnxruntime/torchaudio
        pass

    core.Qwen3TTSTokenizerV1Config = _V1Stub
    core.Qwen3TTSTokenizerV1Model = _V1Stub
    core.Qwen3TTSTokenizerV2Config = ctok.Qwen3TTSTokenizerV2Config
    core.Qwen3TTSTokenizerV2Model = mtok.Qwen3TTSTokenizerV2Model
    cfg = importlib.import_module("qwen_tts.core.models.configuration_qwen3_tts")
    mdl = importlib.import_module("qwen_tts.core.models.modeling_qwen3_tts")
    # Patch 3 in every namespace that imported the mask factories by name.
    for mod in (mdl, mtok):
        mod.create_causal_mask = _make_mask_fn(False)
        mod.create_sliding_window_causal_mask = _make_mask_fn(True)
    del tmask
    # Patch 6
    mdl.Qwen3TTSTalkerForConditionalGeneration.forward = _inject_cache_position(
        mdl.Qwen3TTSTalkerForConditionalGeneration.forward)
    mdl.Qwen3TTSTalkerCodePredictorModelForConditionalGeneration.forward = _inject_cache_position(
        mdl.Qwen3TTSTalkerCodePredictorModelForConditionalGeneration.forward)
    _loaded["mods"] = (mdl, cfg, mtok, ctok)
    return _loaded["mods"]
