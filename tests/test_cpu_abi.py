"""CPU-only: the C-ABI library loads and exports every symbol declared in include/qwen3tts_amd.h."""
import os
import re

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_declared_symbol():
    from qwen_tts import _hip
    L = _hip.load_library()
    hdr = open(os.path.join(REPO, "include", "qwen3tts_amd.h")).read()
    declared = set(re.findall(r"\b(?:int|long long) (qt_\w+)\(", hdr))
    assert declared == set(_hip.EXPORTS)
    for name in declared:
        assert hasattr(L, name), name


def test_qwen2_bpe_files_are_used(tmp_path):
    """A checkpoint directory holding a Qwen2-style BPE tokenizer (tokenizer_config.json + vocab.json /
    merges.txt, as written by save_pretrained) is tokenised by that tokenizer, special tokens included
    (the reference loads it via AutoProcessor, W:103-108); without the files the stand-in is used."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "qwen3-tts_amd"))
    from tokenizers import Tokenizer, models, pre_tokenizers, trainers, decoders
    from transformers import PreTrainedTokenizerFast
    from qwen_tts.text import FallbackProcessor, load_processor
    tk = Tokenizer(models.BPE())
    tk.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tk.decoder = decoders.ByteLevel()
    tr = trainers.BpeTrainer(vocab_size=300, special_tokens=["<|im_start|>", "<|im_end|>"],
                             initial_alphabet=pre_tokenizers.ByteLevel.alphabet())
    tk.train_from_iterator(["hello world, this is a voice clone test", "assistant user text"] * 20, tr)
    hf = PreTrainedTokenizerFast(tokenizer_object=tk)
    hf.add_special_tokens({"additional_special_tokens": ["<|im_start|>", "<|im_end|>"]})
    hf.save_pretrained(str(tmp_path))
    assert os.path.exists(tmp_path / "tokenizer_config.json")
    proc = load_processor(str(tmp_path))
    text = "<|im_start|>assistant\nhello world<|im_end|>\n"
    ids = proc(text=text)["input_ids"]
    assert ids.shape[0] == 1 and ids[0].tolist() == hf(text)["input_ids"]
    assert ids[0, 0].item() == hf.convert_tokens_to_ids("<|im_start|>")
    assert isinstance(load_processor(str(tmp_path / "missing")), FallbackProcessor)
