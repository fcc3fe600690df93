"""CPU-only: the C-ABI library loads and exports every symbol declared in include/qwen3tts_amd.h."""
import os
import re

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_declared_symbol():
    from qwen_tts import _hip
    L = _hip.load_library()
    hdr = open(os.path.join(REPO, "include", "qwen3tts_amd.h")).read()
    declared = set(re.findall(r"\b(?:int|long long|const char\*) (qt_\w+)\(", hdr))
    assert declared == set(_hip.EXPORTS)
    for name in declared:
        assert hasattr(L, name), name
    # the library is the build of the sources in this tree (content digest, not mtime)
    assert _hip.BUILD_ID == _hip.source_digest()


def test_qwen2_bpe_files_are_used(tmp_path):
    """A checkpoint directory holding a Qwen2-style BPE tokenizer (tokenizer_config.json + vocab.json /
    merges.txt, as written by save_pretrained) is tokenised by that tokenizer, special tokens included
    (the reference loads it via AutoProcessor, W:103-108); without the files only the packaged presets fall back
    to the stand-in."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "qwen3-tts_amd"))
    from cases import write_test_tokenizer
    from qwen_tts.text import FallbackProcessor, load_processor
    hf = write_test_tokenizer(tmp_path)
    assert os.path.exists(tmp_path / "tokenizer_config.json")
    proc = load_processor(str(tmp_path))
    text = "<|im_start|>assistant\nhello world<|im_end|>\n"
    ids = proc(text=text)["input_ids"]
    assert ids.shape[0] == 1 and ids[0].tolist() == hf(text)["input_ids"]
    assert ids[0, 0].item() == hf.convert_tokens_to_ids("<|im_start|>")
    # the stand-in is reserved for the packaged synthetic presets; a real checkpoint dir without tokenizer
    # files is an error, not a silent hash tokenizer
    from qwen_tts.weights import resolve_path
    import pytest
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        assert isinstance(load_processor(resolve_path("synthetic:tiny-customvoice")), FallbackProcessor)
    (tmp_path / "ckpt").mkdir()
    with pytest.raises(FileNotFoundError, match="tokenizer"):
        load_processor(str(tmp_path / "ckpt"))


def test_hub_ids_map_to_matching_presets():
    """Every hub id resolves to a preset of its own size and model type (0.6B-Base is not the 1.7B preset)."""
    import json
    import warnings
    from qwen_tts.weights import HUB_ALIASES, resolve_path
    for hub in HUB_ALIASES:
        if "tokenizer" in hub:
            continue
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            d = resolve_path(hub)
        cfg = json.load(open(os.path.join(d, "config.json")))
        size = "0b6" if "0.6b" in hub else "1b7"
        mtype = {"customvoice": "custom_voice", "voicedesign": "voice_design", "base": "base"}[hub.rsplit("-", 1)[1]]
        assert cfg["tts_model_size"] == size and cfg["tts_model_type"] == mtype, hub
        assert cfg["talker_config"]["hidden_size"] == (1024 if size == "0b6" else 2048), hub
        if mtype == "base":
            assert cfg["speaker_encoder_config"]["enc_dim"] == cfg["talker_config"]["hidden_size"], hub
