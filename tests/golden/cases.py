"""Golden-case definitions shared by the fixture generator (make_golden.py) and the parity tests.

Pure data/helpers: no reference import, so the GPU-box tests can rebuild the exact same inputs.
Synthetic token ids follow the wrapper templates of qwen_tts/inference/qwen3_tts_model.py:269-276
(`<|im_start|>assistant\n{text}<|im_end|>\n<|im_start|>assistant\n` etc.; no BPE offline).
"""
import numpy as np
import torch


def text_ids(n, seed):
    g = np.random.default_rng([seed, 7])
    body = g.integers(1000, 150000, n).tolist()
    return torch.tensor([[151644, 77091, 198] + body + [151645, 198, 151644, 77091, 198]], dtype=torch.long)


def instruct_ids(n, seed):
    g = np.random.default_rng([seed, 11])
    return torch.tensor([[151644, 872, 198] + g.integers(1000, 150000, n).tolist() + [151645, 198]],
                        dtype=torch.long)


def ref_text_ids(n, seed):
    g = np.random.default_rng([seed, 13])
    return torch.tensor([[151644, 77091, 198] + g.integers(1000, 150000, n).tolist() + [151645, 198]],
                        dtype=torch.long)


def talker_cases():
    """Prompt layouts covering SURVEY.md §8a G1/G2 and Appendix A (each case = kwargs of generate)."""
    return {
        "cv_b1_nonstream": dict(texts=[9], languages=["english"], speakers=["vivian"], non_streaming_mode=True,
                                max_new_tokens=13),
        "cv_b2_stream_dialect": dict(texts=[12, 5], languages=["chinese", "auto"], speakers=["eric", "ryan"],
                                     non_streaming_mode=False, max_new_tokens=16),
        "cv_b3_auto_nospk": dict(texts=[7, 3, 10], languages=["auto", "english", "japanese"],
                                 speakers=["", None, "dylan"], non_streaming_mode=False, max_new_tokens=12),
        "vd_b2_instruct": dict(texts=[6, 11], languages=["english", "auto"], speakers=None, instruct=[8, 0],
                               non_streaming_mode=True, max_new_tokens=10),
        "cv_b2_sample": dict(texts=[8, 4], languages=["english", "chinese"], speakers=["vivian", "ryan"],
                             non_streaming_mode=False, max_new_tokens=10, do_sample=True,
                             subtalker_dosample=True, seed=77),
        "icl_b2": dict(texts=[6, 9], languages=["english", "auto"], speakers=None, non_streaming_mode=False,
                       max_new_tokens=10, icl=[(5, 7, True, False), (12, 4, False, True)]),
        "icl_b1_nonstream": dict(texts=[5], languages=["english"], speakers=None, non_streaming_mode=True,
                                 max_new_tokens=8, icl=[(4, 6, True, False)]),
    }


FULL_SPEAKERS = ["vivian", "ryan", "serena", "aiden", "eric", "dylan", "sohee", "ono_anna"]


def full_cases():
    """Production-shape greedy cases (BASELINE.json configs[1] / configs[2]): reference codes, per-pick
    top-2 margins and first hidden states are in tests/golden/full_<key>.npz.  `idx` seeds the token ids."""
    return {
        # configs[2]: 1.7B CustomVoice, B=8 x 200-token prompts, streaming text (trailing text fed per frame)
        "cv17_b8_stream": dict(preset="1.7b-customvoice", idx=60, texts=[200] * 8, languages=["english"] * 8,
                               speakers=FULL_SPEAKERS, non_streaming_mode=False, max_new_tokens=33),
        # configs[2] at the bench's length: 1.7B CustomVoice, 2 rows x 200 / 150-token prompts, streaming text, 256
        # frames (talker caches up to ~460 keys: the decode attention's length range in bench.py)
        "cv17_b2_long": dict(preset="1.7b-customvoice", idx=64, texts=[200, 150], languages=["english", "chinese"],
                             speakers=FULL_SPEAKERS[:2], non_streaming_mode=False, max_new_tokens=257),
        # the long-cache route: 1.7B CustomVoice, 2 rows x 800 / 1000-token texts, NON-streaming (the whole text in the
        # prompt), 48 frames -- talker caches of ~810-1060 keys, so every frame runs the split-KV decode attention
        # (talker.attn_nsplit: 2 splits from 768 keys) and the refill-free frame graph of that split factor
        "cv17_b2_longctx": dict(preset="1.7b-customvoice", idx=65, texts=[800, 1000], languages=["english", "auto"],
                                speakers=FULL_SPEAKERS[2:4], non_streaming_mode=True, max_new_tokens=49),
        # the 4-split route: 2 rows x ~2,070 / 2,100-token texts, non-streaming, 16 frames -- talker caches of ~2,080-2,130
        # keys, past talker.attn_nsplit's 2,048-key bound, so every frame runs the 4-split decode attention (the wrapper
        # allows 2,048 new tokens and the model 4,096: W:329, M:2031)
        "cv17_b2_longctx4": dict(preset="1.7b-customvoice", idx=66, texts=[2060, 2100], languages=["english", "auto"],
                                 speakers=FULL_SPEAKERS[4:6], non_streaming_mode=True, max_new_tokens=17),
        # configs[1]: 0.6B CustomVoice, 1 utterance of 120 text tokens, non-streaming (Identity small_to_mtp, M:1174)
        "cv06_b1_nonstream": dict(preset="0.6b-customvoice", idx=61, texts=[120], languages=["english"],
                                  speakers=["vivian"], non_streaming_mode=True, max_new_tokens=49),
        # configs[3] shape: 1.7B VoiceDesign, mixed-length texts and instructs (one row without), left-padded batch
        "vd17_b4_instruct": dict(preset="1.7b-voicedesign", idx=62, texts=[60, 25, 110, 40], instruct=[30, 12, 0, 45],
                                 languages=["english", "chinese", "auto", "japanese"], speakers=None,
                                 non_streaming_mode=True, max_new_tokens=25),
        # configs[4] shape: 1.7B-Base voice clone, one ICL row (40-token reference text, 38 reference frames) and one
        # x-vector-only row, streaming text (the voice-clone wrapper's default)
        "base17_b2_clone": dict(preset="1.7b-base", idx=63, texts=[50, 30], languages=["english", "auto"], speakers=None,
                                icl=[(40, 38, True, False), (20, 25, False, True)], non_streaming_mode=False,
                                max_new_tokens=25),
    }


def margins_grid(flat, B, n_tokens, groups=16):
    """oracle.generate(record_margins=True) logs the top-2 margin of every greedy pick in generation order: per talker
    step the B cb0 picks, then (if the loop continues) the code predictor's 15 x B picks.  Returns [B, frames, 16] in
    the layout of the codes (frame f = cb0 of step f + the CP codes drawn during step f+1)."""
    a = np.asarray(flat, dtype=np.float32)
    frames = n_tokens - 1
    a = a[:frames * groups * B].reshape(frames, groups, B)
    return np.ascontiguousarray(a.transpose(2, 0, 1))


def first_divergence(got, ref, margins, tol):
    """Per row: first (frame, group) in generation order where `got` differs from `ref`.  Returns a list of
    (row, flat index or None, reference margin there)."""
    out = []
    for b, (g, r) in enumerate(zip(got, ref)):
        n = min(g.shape[0], r.shape[0])
        d = np.flatnonzero((np.asarray(g[:n]) != np.asarray(r[:n])).reshape(-1))
        if d.size == 0:
            out.append((b, None, None))
        else:
            i = int(d[0])
            out.append((b, i, float(margins[b].reshape(-1)[i])))
    return out


def make_inputs(case, idx, H):
    ids = [text_ids(n, 100 * idx + j) for j, n in enumerate(case["texts"])]
    ins = None
    if "instruct" in case:
        ins = [instruct_ids(n, 200 * idx + j) if n else None for j, n in enumerate(case["instruct"])]
    vcp, ref_ids = None, None
    if "icl" in case:
        g = np.random.default_rng([idx, 17])
        vcp = dict(ref_code=[], ref_spk_embedding=[], x_vector_only_mode=[], icl_mode=[])
        ref_ids = []
        for j, (nref, ncode, icl, xvec) in enumerate(case["icl"]):
            vcp["ref_code"].append(torch.tensor(g.integers(0, 2048, (ncode, 16)), dtype=torch.long) if icl else None)
            vcp["ref_spk_embedding"].append(torch.tensor(0.02 * g.standard_normal(H), dtype=torch.float32))
            vcp["x_vector_only_mode"].append(xvec)
            vcp["icl_mode"].append(icl)
            ref_ids.append(ref_text_ids(nref, 300 * idx + j))
    return ids, ins, vcp, ref_ids


def gen_kwargs(case):
    return dict(max_new_tokens=case["max_new_tokens"], do_sample=case.get("do_sample", False),
                subtalker_dosample=case.get("subtalker_dosample", False), top_k=50, top_p=1.0, temperature=0.9,
                subtalker_top_k=50, subtalker_top_p=1.0, subtalker_temperature=0.9, repetition_penalty=1.05)




def ref_audio(n, seed):
    """Deterministic 24 kHz reference clip (voice-clone front end cases): two partials with a slow tremolo
    plus seeded noise, float32 in about [-0.45, 0.45].  Pure float64 numpy arithmetic, so the GPU box
    rebuilds bit-identical inputs."""
    t = np.arange(n, dtype=np.float64) / 24000.0
    g = np.random.default_rng([seed, 23])
    f0 = 110.0 + 20.0 * (seed % 7)
    x = 0.25 * np.sin(2 * np.pi * f0 * t) * (1.0 + 0.5 * np.sin(2 * np.pi * 3.0 * t))
    x += 0.1 * np.sin(2 * np.pi * 7.3 * f0 * t + 0.3)
    x += 0.05 * g.standard_normal(n)
    return x.astype(np.float32)


def frontend_cases():
    """Encoder (Mimi) batches and speaker-encoder clips: lengths in samples at 24 kHz."""
    return {
        "tiny": dict(enc={"single": [31234], "batch": [40000, 17000], "exact": [3840], "short": [1000]},
                     spk=[24000, 7777]),
        "full": dict(enc={"single": [72000], "batch": [50000, 72000]}, spk=[72000]),
    }


def write_test_tokenizer(path):
    """A small byte-level BPE tokenizer saved in the Hugging Face layout of a Qwen2 checkpoint
    (tokenizer_config.json + tokenizer.json, special tokens included): real checkpoint directories must carry
    tokenizer files (the hash stand-in is reserved for the packaged presets).  Returns the tokenizer."""
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers, trainers
    from transformers import PreTrainedTokenizerFast
    tk = Tokenizer(models.BPE())
    tk.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tk.decoder = decoders.ByteLevel()
    tr = trainers.BpeTrainer(vocab_size=300, special_tokens=["<|im_start|>", "<|im_end|>"],
                             initial_alphabet=pre_tokenizers.ByteLevel.alphabet())
    tk.train_from_iterator(["hello world, this is a voice clone test", "assistant user text"] * 20, tr)
    hf = PreTrainedTokenizerFast(tokenizer_object=tk)
    hf.add_special_tokens({"additional_special_tokens": ["<|im_start|>", "<|im_end|>"]})
    hf.save_pretrained(str(path))
    return hf
