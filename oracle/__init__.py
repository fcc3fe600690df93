"""Oracle: CPU fp32 restatement of the reference hot path (talker + code predictor + HF-4.57
generation loop + 12 Hz codec decoder).

TEST INFRASTRUCTURE.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package, and only as the checker / CPU baseline -- never as the thing measured or shipped.  The
product package (qwen3-tts_amd/qwen_tts) never imports it and fails loudly when its HIP library is
missing.

Parity pin: tests/test_oracle_golden.py checks this restatement against golden vectors produced by the
reference itself (imported here with the shims of tests/golden/ref_shim.py; generator
tests/golden/make_golden.py).
"""
import json
import os

from .talker import TalkerOracle, build_prompts, generate, talker_param_specs  # noqa: F401
from .codec import CodecOracle, codec_param_specs, tokenizer_decode  # noqa: F401
from .weights import synth_param, synth_state_dict  # noqa: F401

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PRESETS = os.path.join(REPO, "qwen3-tts_amd", "qwen_tts", "configs")


def load_preset(name):
    """(model config dict, codec config dict) of a synthetic checkpoint preset (JSON data files)."""
    d = os.path.join(PRESETS, name)
    with open(os.path.join(d, "config.json")) as f:
        cfg = json.load(f)
    with open(os.path.join(d, "speech_tokenizer", "config.json")) as f:
        ccfg = json.load(f)
    return cfg, ccfg
