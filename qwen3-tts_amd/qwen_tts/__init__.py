"""qwen_tts (MI355X build): drop-in for the reference's `qwen_tts` package hot path.

`from qwen_tts import Qwen3TTSModel, Qwen3TTSTokenizer` exactly as the reference examples do
(reference: qwen_tts/__init__.py:21-22).  Compute runs through libqwen3tts_amd.so (hand-written gfx950
HIP kernels); there is no CPU fallback.
"""
__version__ = "0.0.4+mi355x"

from .inference.qwen3_tts_model import (Qwen3TTSModel, VoiceClonePromptItem, load_voice_clone_prompt,  # noqa: E402,F401
                                       save_voice_clone_prompt)
from .inference.qwen3_tts_tokenizer import Qwen3TTSTokenizer  # noqa: E402,F401

__all__ = ["__version__", "Qwen3TTSModel", "Qwen3TTSTokenizer", "VoiceClonePromptItem", "load_voice_clone_prompt",
           "save_voice_clone_prompt"]
