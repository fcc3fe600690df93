"""The reference's example entry points, replayed through the drop-in wrapper (`qwen_tts.Qwen3TTSModel`):
examples/test_model_12hz_custom_voice.py:38-66, examples/test_model_12hz_voice_design.py:38-66 and
examples/test_model_12hz_base.py:95-188 -- the same call sequences, texts, languages, speakers and instructs -- on the
tiny presets in fp32 parity mode.  Two deliberate changes, so the output is comparable: greedy decoding
(do_sample=False, subtalker_dosample=False; the examples sample, whose RNG stream is device-specific -- sampling is
checked at distribution level in test_gpu_parity.py) and max_new_tokens=10.  Reference audio for voice clone is a
synthetic 24 kHz clip (the examples download theirs).

Every result is compared with the oracle (prompt assembly M:2068-2269 + the HF-4.57 loop + codec decode Z:259-365,
pinned to the reference itself by tests/test_oracle_golden.py) on the ids the wrapper's tokenizer produced: codes
bit-exact, PCM within 2e-4.  The 0.6B instruct drop (`tts_model_size in "0b6"`, W:799) is exercised on a tiny model
given the 0.6B size tag.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

GREEDY = dict(do_sample=False, subtalker_dosample=False, max_new_tokens=10)
PCM_TOL = 2e-4


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


_CACHE = {}


def _setup(preset):
    """(wrapper, oracle talker, oracle codec, cfg) on the oracle's seeded weights."""
    if preset in _CACHE:
        return _CACHE[preset]
    from oracle import (CodecOracle, TalkerOracle, codec_param_specs, load_preset, synth_state_dict,
                        talker_param_specs)
    from oracle.encoder import encoder_param_specs
    from oracle.speaker import speaker_param_specs
    from qwen_tts import Qwen3TTSModel
    _dev()
    cfg, ccfg = load_preset(preset)
    specs = talker_param_specs(cfg) + (speaker_param_specs(cfg) if cfg.get("tts_model_type") == "base" else [])
    Wn = synth_state_dict(specs)
    CWn = synth_state_dict(codec_param_specs(ccfg) + encoder_param_specs(ccfg))
    tts = Qwen3TTSModel.from_pretrained(f"synthetic:{preset}", dtype=torch.float32,
                                        weights={k: torch.from_numpy(v) for k, v in Wn.items()},
                                        codec_weights={k: torch.from_numpy(v) for k, v in CWn.items()})
    out = (tts, TalkerOracle(cfg, Wn), CodecOracle(ccfg, CWn), cfg)
    _CACHE.clear()
    _CACHE[preset] = out
    return out


def _ids(tts, texts, build):
    return [None if not t else tts._tokenize_texts([build(t)])[0] for t in texts]


def _oracle(o, co, input_ids, languages, speakers=None, instruct_ids=None, non_streaming_mode=True, vcp=None,
            ref_ids=None):
    """Oracle generate + the wrapper's decode step (W:612-631 for voice clone: decode cat(ref_code, codes), cut the
    reference part proportionally)."""
    from oracle import build_prompts, generate, tokenizer_decode
    emb, mask, trail, pad = build_prompts(o, input_ids, languages, speakers, instruct_ids, non_streaming_mode, vcp,
                                          ref_ids)
    res = generate(o, emb, mask, trail, pad, max_new_tokens=GREEDY["max_new_tokens"], do_sample=False,
                   subtalker_dosample=False, repetition_penalty=1.05)
    refs = vcp["ref_code"] if vcp is not None else [None] * len(res.codes)
    dec = [c if r is None else torch.cat([torch.as_tensor(r).cpu().long(), c], 0) for c, r in zip(res.codes, refs)]
    wavs = tokenizer_decode(co, [c.numpy() for c in dec])
    out = []
    for w, r, d in zip(wavs, refs, dec):
        if r is not None:
            w = w[int(int(r.shape[0]) / max(int(d.shape[0]), 1) * w.shape[0]):]
        out.append(w)
    return res.codes, out


def _same_pcm(got, ref, label):
    assert len(got) == len(ref), label
    for i, (a, b) in enumerate(zip(got, ref)):
        assert a.shape == b.shape, (label, i, a.shape, b.shape)
        np.testing.assert_allclose(a, b, atol=PCM_TOL, rtol=0, err_msg=f"{label}[{i}]")


CV_TEXT = "其实我真的有发现，我是一个特别善于观察别人情绪的人。"


def test_example_custom_voice():
    """examples/test_model_12hz_custom_voice.py:38-66: single with instruct, then a batch whose first instruct is
    empty (no instruct row for it)."""
    tts, o, co, cfg = _setup("tiny-customvoice")
    wavs, sr = tts.generate_custom_voice(text=CV_TEXT, language="Chinese", speaker="Vivian",
                                         instruct="用特别愤怒的语气说", **GREEDY)
    assert sr == 24000 and len(wavs) == 1
    ids = _ids(tts, [CV_TEXT], tts._build_assistant_text)
    ins = _ids(tts, ["用特别愤怒的语气说"], tts._build_instruct_text)
    _, ref = _oracle(o, co, ids, ["Chinese"], ["Vivian"], ins)
    _same_pcm(wavs, ref, "custom_voice single")

    texts = [CV_TEXT, "She said she would be here by noon."]
    languages, speakers, instructs = ["Chinese", "English"], ["Vivian", "Ryan"], ["", "Very happy."]
    wavs, sr = tts.generate_custom_voice(text=texts, language=languages, speaker=speakers, instruct=instructs,
                                         **GREEDY)
    ids = _ids(tts, texts, tts._build_assistant_text)
    ins = _ids(tts, instructs, tts._build_instruct_text)
    assert ins[0] is None
    _, ref = _oracle(o, co, ids, languages, speakers, ins)
    _same_pcm(wavs, ref, "custom_voice batch")


def test_example_custom_voice_0b6_drops_instruct():
    """W:799: a model whose tts_model_size is in "0b6" ignores instruct (the 0.6B CustomVoice checkpoints): the
    single example call with its instruct gives exactly the no-instruct output, and the oracle agrees."""
    tts, o, co, cfg = _setup("tiny-customvoice")
    size = tts.model.tts_model_size
    try:
        tts.model.tts_model_size = "0b6"
        a, _ = tts.generate_custom_voice(text=CV_TEXT, language="Chinese", speaker="Vivian",
                                         instruct="用特别愤怒的语气说", **GREEDY)
        b, _ = tts.generate_custom_voice(text=CV_TEXT, language="Chinese", speaker="Vivian", **GREEDY)
    finally:
        tts.model.tts_model_size = size
    np.testing.assert_array_equal(a[0], b[0])
    ids = _ids(tts, [CV_TEXT], tts._build_assistant_text)
    _, ref = _oracle(o, co, ids, ["Chinese"], ["Vivian"], None)
    _same_pcm(a, ref, "custom_voice 0b6")


def test_example_voice_design():
    """examples/test_model_12hz_voice_design.py:38-66: single, then a batch of two (instruct prepended, no speaker)."""
    tts, o, co, cfg = _setup("tiny-voicedesign")
    t1 = "哥哥，你回来啦，人家等了你好久好久了，要抱抱！"
    i1 = "体现撒娇稚嫩的萝莉女声，音调偏高且起伏明显，营造出黏人、做作又刻意卖萌的听觉效果。"
    wavs, sr = tts.generate_voice_design(text=t1, language="Chinese", instruct=i1, **GREEDY)
    _, ref = _oracle(o, co, _ids(tts, [t1], tts._build_assistant_text), ["Chinese"], None,
                     _ids(tts, [i1], tts._build_instruct_text))
    _same_pcm(wavs, ref, "voice_design single")
    texts = [t1, "It's in the top drawer... wait, it's empty? No way, that's impossible! I'm sure I put it there!"]
    languages = ["Chinese", "English"]
    instructs = [i1, "Speak in an incredulous tone, but with a hint of panic beginning to creep into your voice."]
    wavs, sr = tts.generate_voice_design(text=texts, language=languages, instruct=instructs, **GREEDY)
    _, ref = _oracle(o, co, _ids(tts, texts, tts._build_assistant_text), languages, None,
                     _ids(tts, instructs, tts._build_instruct_text))
    _same_pcm(wavs, ref, "voice_design batch")
    with pytest.raises(ValueError):
        tts.generate_custom_voice(text=t1, speaker="Vivian")  # wrong model type (W:788-794)


@pytest.mark.parametrize("xvec_only", [False, True])
def test_example_voice_clone(xvec_only):
    """examples/test_model_12hz_base.py:95-188 for one x_vector_only_mode: cases 1/1b (prompt single, synth single;
    direct and via create_voice_clone_prompt), 2/2b (prompt single, synth batch), 3/3b (prompt batch, synth batch).
    Direct and prompt-then-generate agree exactly; each equals the oracle given the same voice-clone prompt."""
    from cases import ref_audio
    tts, o, co, cfg = _setup("tiny-base")
    ra1, ra2 = (ref_audio(31234, 5), 24000), (ref_audio(26000, 6), 24000)
    rt1 = "Okay. Yeah. I resent you. I love you. I respect you. But you know what? You blew it! And thanks to you."
    rt_batch = [rt1, "甚至出现交易几乎停滞的情况。"]
    s1 = "Good one. Okay, fine, I'm just gonna leave this sock monkey here. Goodbye."
    s_batch = [s1, CV_TEXT]
    l_batch = ["Chinese", "English"]

    def check(wavs, texts, languages, items, label):
        vcp = tts._prompt_items_to_voice_clone_prompt(items if len(items) == len(texts) else items * len(texts))
        vcp = {k: [x.cpu() if isinstance(x, torch.Tensor) else x for x in v] for k, v in vcp.items()}
        ref_texts = [it.ref_text for it in (items if len(items) == len(texts) else items * len(texts))]
        ref_ids = [None if not rt else tts._tokenize_texts([tts._build_ref_text(rt)])[0] for rt in ref_texts]
        _, ref = _oracle(o, co, _ids(tts, texts, tts._build_assistant_text), languages, None, None,
                         non_streaming_mode=False, vcp=vcp, ref_ids=ref_ids)
        _same_pcm(wavs, ref, label)

    # case 1 / 1b
    a, sr = tts.generate_voice_clone(text=s1, language="Auto", ref_audio=ra1, ref_text=rt1, x_vector_only_mode=xvec_only,
                                     **GREEDY)
    items = tts.create_voice_clone_prompt(ref_audio=ra1, ref_text=rt1, x_vector_only_mode=xvec_only)
    b, _ = tts.generate_voice_clone(text=s1, language="Auto", voice_clone_prompt=items, **GREEDY)
    _same_pcm(a, b, "case1 direct vs prompt")
    check(b, [s1], ["Auto"], items, "case1")
    # case 2 / 2b
    a, _ = tts.generate_voice_clone(text=s_batch, language=l_batch, ref_audio=ra1, ref_text=rt1,
                                    x_vector_only_mode=xvec_only, **GREEDY)
    b, _ = tts.generate_voice_clone(text=s_batch, language=l_batch, voice_clone_prompt=items, **GREEDY)
    _same_pcm(a, b, "case2 direct vs prompt")
    check(b, s_batch, l_batch, items, "case2")
    # case 3 / 3b
    a, _ = tts.generate_voice_clone(text=s_batch, language=l_batch, ref_audio=[ra1, ra2], ref_text=rt_batch,
                                    x_vector_only_mode=[xvec_only, xvec_only], **GREEDY)
    items3 = tts.create_voice_clone_prompt(ref_audio=[ra1, ra2], ref_text=rt_batch,
                                           x_vector_only_mode=[xvec_only, xvec_only])
    b, _ = tts.generate_voice_clone(text=s_batch, language=l_batch, voice_clone_prompt=items3, **GREEDY)
    _same_pcm(a, b, "case3 direct vs prompt")
    check(b, s_batch, l_batch, items3, "case3")
