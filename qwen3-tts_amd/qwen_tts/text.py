"""Text processor stand-in for the Qwen2 BPE processor (qwen_tts/inference/qwen3_tts_model.py:278-285).

A real `tokenizer.json` in the checkpoint dir is used through the `tokenizers` library when present.
Offline there is none, so the fallback maps text deterministically to ids in
[1000, 150000) while reproducing the special-token layout the reference slices on
(`[:3]` role tokens, `[3:-5]` text, `[-5:]` suffix; M:2178-2231).
"""
from __future__ import annotations

import os
import re
import zlib

import torch

SPECIAL = {"<|im_start|>": 151644, "<|im_end|>": 151645, "<tts_pad>": 151671, "<tts_text_bos>": 151672,
           "<tts_text_eod>": 151673}
WORDS = {"assistant": 77091, "user": 872, "\n": 198}
_SPLIT = re.compile(r"(<\|im_start\|>|<\|im_end\|>|\n)")


class FallbackProcessor:
    def __call__(self, text, return_tensors="pt", padding=True):
        ids = []
        for part in _SPLIT.split(text):
            if not part:
                continue
            if part in SPECIAL:
                ids.append(SPECIAL[part])
            elif part in WORDS:
                ids.append(WORDS[part])
            elif ids and ids[-1] == SPECIAL["<|im_start|>"] and part in WORDS:
                ids.append(WORDS[part])
            else:
                for w in re.findall(r"\w+|[^\w\s]|\s+", part):
                    if w in WORDS:
                        ids.append(WORDS[w])
                    else:
                        ids.append(1000 + zlib.crc32(w.encode("utf-8")) % 149000)
        return {"input_ids": torch.tensor([ids], dtype=torch.long)}


def load_processor(path: str):
    """The checkpoint's Qwen2 BPE tokenizer when its files are present (the reference loads it through
    AutoProcessor, W:103-108): `tokenizer_config.json` + `vocab.json` / `merges.txt` (or `tokenizer.json`) via
    transformers' AutoTokenizer from the local directory; a bare `tokenizer.json` via the `tokenizers` library.
    The deterministic stand-in above is used only for the packaged synthetic presets: a real checkpoint
    directory without tokenizer files raises FileNotFoundError instead of silently hashing text."""
    if os.path.exists(os.path.join(path, "tokenizer_config.json")) and (
            os.path.exists(os.path.join(path, "vocab.json")) or os.path.exists(os.path.join(path, "tokenizer.json"))):
        from transformers import AutoTokenizer
        hf = AutoTokenizer.from_pretrained(path, local_files_only=True)

        class _HF:
            tokenizer = hf

            def __call__(self, text, return_tensors="pt", padding=True):
                return {"input_ids": torch.tensor([hf(text)["input_ids"]], dtype=torch.long)}

        return _HF()
    tj = os.path.join(path, "tokenizer.json")
    if os.path.exists(tj):
        from tokenizers import Tokenizer
        tok = Tokenizer.from_file(tj)

        class _P:
            def __call__(self, text, return_tensors="pt", padding=True):
                return {"input_ids": torch.tensor([tok.encode(text).ids], dtype=torch.long)}

        return _P()
    from .weights import is_preset_dir
    if is_preset_dir(path):
        return FallbackProcessor()
    raise FileNotFoundError(
        f"no Qwen2 BPE tokenizer in {path!r}: expected tokenizer_config.json + vocab.json/merges.txt, or "
        "tokenizer.json (the stand-in tokenizer is reserved for the packaged synthetic presets)")
