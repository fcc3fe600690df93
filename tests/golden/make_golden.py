"""Generate golden vectors by running the REFERENCE (`/root/reference/qwen_tts`) in this container.

    python tests/golden/make_golden.py            # tiny talker + tiny/full codec fixtures
    python tests/golden/make_golden.py --full     # + full ASSUMED-dim 1.7B greedy codes (slow, ~16 GB RAM)

Test infrastructure only: needs /root/reference (absent on the GPU box).  The reference is imported
through tests/golden/ref_shim.py (transformers-5.15 -> 4.57 patches).  Weights are the
seeded synthetic ones of oracle/weights.py loaded into the reference modules by state_dict name, so the
oracle and the HIP path can regenerate identical weights without the fixture storing them.

Fixtures written (inputs + expected outputs only):
  tiny_talker.npz   greedy / sampled / EOS / ICL generate() codes for several prompt layouts
  codec_*.npz       12 Hz decoder PCM for fixed codes (single, right-padded batch, chunked > 300 frames)
  param_specs.json  reference state_dict names and shapes per preset (the checkpoint key contract)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, REPO)

import ref_shim  # noqa: E402
from cases import frontend_cases, gen_kwargs, make_inputs, ref_audio, talker_cases  # noqa: E402,F401
from oracle import load_preset  # noqa: E402
from oracle.weights import synth_param  # noqa: E402

SEED = 1234


def _eagerize(c):
    c._attn_implementation = "eager"
    c.pad_token_id = None


def build_ref_model(name, seed=SEED, meta=False):
    mdl, cfgm, _, _ = ref_shim.load_reference()
    cfg, _ = load_preset(name)
    config = cfgm.Qwen3TTSConfig(**json.loads(json.dumps(cfg)))
    for c in (config, config.talker_config, config.talker_config.code_predictor_config):
        _eagerize(c)
    if meta:
        with torch.device("meta"):
            return mdl.Qwen3TTSForConditionalGeneration(config), cfg
    torch.manual_seed(0)
    model = mdl.Qwen3TTSForConditionalGeneration(config).eval()
    sd = model.state_dict()
    new = {k: torch.from_numpy(synth_param(k, v.shape, seed)) for k, v in sd.items()}
    model.load_state_dict(new)
    return model, cfg


def build_ref_codec(name, seed=SEED, meta=False):
    _, _, mtok, ctok = ref_shim.load_reference()
    _, ccfg = load_preset(name)
    config = ctok.Qwen3TTSTokenizerV2Config(**json.loads(json.dumps(ccfg)))
    dc = config.decoder_config
    _eagerize(dc)
    ctx = torch.device("meta") if meta else torch.device("cpu")
    with ctx:
        dec = mtok.Qwen3TTSTokenizerV2Decoder(dc).eval()
    if meta:
        return dec, ccfg
    sd = dec.state_dict()
    dec.load_state_dict({k: torch.from_numpy(synth_param("decoder." + k, v.shape, seed)) for k, v in sd.items()})
    return dec, ccfg


class _CodecModelView:
    """The attributes Qwen3TTSTokenizerV2Model.decode reads (K:992-1022), so the reference method itself runs."""

    def __init__(self, decoder, ccfg):
        class C:
            return_dict = True
        self.config = C()
        self.decoder = decoder
        self.decode_upsample_rate = ccfg["decode_upsample_rate"]


def ref_codec_decode(dec, ccfg, codes_list):
    """Qwen3TTSTokenizer.decode list path (Z:259-365) on top of the reference V2Model.decode."""
    _, _, mtok, _ = ref_shim.load_reference()
    codes = [torch.as_tensor(c, dtype=torch.long) for c in codes_list]
    padded = torch.nn.utils.rnn.pad_sequence(codes, batch_first=True, padding_value=0)
    with torch.inference_mode():
        out = mtok.Qwen3TTSTokenizerV2Model.decode(_CodecModelView(dec, ccfg), padded, return_dict=True)
    return [w.to(torch.float32).numpy() for w in out.audio_values]


def run_ref_generate(model, case, idx, H):
    ids, ins, vcp, ref_ids = make_inputs(case, idx, H)
    torch.manual_seed(case.get("seed", 0))
    with torch.no_grad():
        codes, hid = model.generate(input_ids=ids, instruct_ids=ins, ref_ids=ref_ids, voice_clone_prompt=vcp,
                                    languages=case["languages"], speakers=case["speakers"],
                                    non_streaming_mode=case["non_streaming_mode"], **gen_kwargs(case))
    return codes, hid


def pack_case(out, key, case, codes, hid):
    out[f"{key}/n"] = np.array(len(codes))
    for j, (c, h) in enumerate(zip(codes, hid)):
        out[f"{key}/codes{j}"] = c.numpy().astype(np.int32)
        out[f"{key}/hidden{j}"] = h.numpy().astype(np.float32)


def make_tiny_talker(preset="tiny-customvoice"):
    model, cfg = build_ref_model(preset)
    H = cfg["talker_config"]["hidden_size"]
    out = {}
    cases = talker_cases()
    for idx, (key, case) in enumerate(cases.items()):
        if key.startswith("vd_"):
            continue  # voice-design preset below (only the wrapper differs; generate() is the same)
        t0 = time.time()
        codes, hid = run_ref_generate(model, case, idx, H)
        pack_case(out, key, case, codes, hid)
        print(f"  {key}: frames {[c.shape[0] for c in codes]} ({time.time() - t0:.1f}s)")
    vd_model, _ = build_ref_model("tiny-voicedesign")
    for idx, (key, case) in enumerate(cases.items()):
        if key.startswith("vd_"):
            codes, hid = run_ref_generate(vd_model, case, idx, H)
            pack_case(out, key, case, codes, hid)
            print(f"  {key}: frames {[c.shape[0] for c in codes]}")
    # EOS case: copy a frequently chosen cb0 row into the EOS row of codec_head so EOS wins the second time
    # that token would be picked (repetition penalty divides the repeated one) -> early, ragged stops.
    eos = cfg["talker_config"]["codec_eos_token_id"]
    key, case = "cv_b2_stream_dialect", cases["cv_b2_stream_dialect"]
    c0 = torch.cat([torch.from_numpy(out[f"{key}/codes{j}"][:, 0]) for j in range(2)])
    vals, counts = torch.unique(c0, return_counts=True)
    donor = int(vals[torch.argmax(counts)])
    with torch.no_grad():
        model.talker.codec_head.weight[eos] = model.talker.codec_head.weight[donor]
    case = dict(case, max_new_tokens=24)
    codes, hid = run_ref_generate(model, case, list(cases).index(key), H)
    pack_case(out, "eos_b2", case, codes, hid)
    out["eos_b2/donor"] = np.array(donor)
    print(f"  eos_b2 (donor {donor}): frames {[c.shape[0] for c in codes]}")
    np.savez_compressed(os.path.join(HERE, "tiny_talker.npz"), **out)


def make_codec(preset, cases, fname, stride=7):
    dec, ccfg = build_ref_codec(preset)
    out = {}
    g = np.random.default_rng(4321)
    for key, lens in cases.items():
        codes = [g.integers(0, 2048, (n, 16)).astype(np.int64) for n in lens]
        codes[0][min(3, lens[0] - 1), 0] = 0  # a legit cb0 == 0 shortens the output (quirk C0-3)
        t0 = time.time()
        wavs = ref_codec_decode(dec, ccfg, codes)
        for j, (c, w) in enumerate(zip(codes, wavs)):
            out[f"{key}/codes{j}"] = c.astype(np.int32)
            out[f"{key}/len{j}"] = np.array(w.shape[0])
            if w.shape[0] > 200_000:  # keep fixtures small: strided samples + checksums for long outputs
                out[f"{key}/stride"] = np.array(stride)
                out[f"{key}/wav{j}_stride"] = w[::stride].copy()
                out[f"{key}/wav{j}_sum"] = np.array([w.astype(np.float64).sum(), (w.astype(np.float64) ** 2).sum()])
            else:
                out[f"{key}/wav{j}"] = w
        print(f"  {fname}:{key} lens {[w.shape[0] for w in wavs]} ({time.time() - t0:.1f}s)")
    np.savez_compressed(os.path.join(HERE, fname), **out)


class _SpeakerModelView:
    """The attributes Qwen3TTSForConditionalGeneration.extract_speaker_embedding reads (M:1940-1954)."""

    def __init__(self, enc):
        self.speaker_encoder = enc
        self.device = torch.device("cpu")
        self.dtype = torch.float32


def make_frontend(preset, kind, fname):
    """Voice-clone front end: reference Qwen3TTSTokenizerV2Model.encode (K:960-990, Mimi from transformers) and
    extract_speaker_embedding (M:1940-1954) on seeded synthetic weights.  librosa is absent: its slaney mel
    filterbank is supplied by oracle.speaker.slaney_mel_filterbank (a restatement; see that module)."""
    from oracle.speaker import slaney_mel_filterbank
    mdl, cfgm, mtok, ctok = ref_shim.load_reference()
    mdl.librosa_mel_fn = lambda sr, n_fft, n_mels, fmin, fmax: slaney_mel_filterbank(sr, n_fft, n_mels, fmin, fmax)
    cfg, ccfg = load_preset(preset)
    cases = frontend_cases()[kind]
    out = {}
    # tokenizer encoder
    config = ctok.Qwen3TTSTokenizerV2Config(**json.loads(json.dumps(ccfg)))
    _eagerize(config.decoder_config)
    torch.manual_seed(0)
    tok = mtok.Qwen3TTSTokenizerV2Model(config).eval()
    sd = tok.state_dict()
    tok.load_state_dict({k: torch.from_numpy(synth_param(k, v.shape, SEED)) for k, v in sd.items()})
    for key, lens in cases["enc"].items():
        wavs = [ref_audio(n, 1000 + 10 * i + n % 97) for i, n in enumerate(lens)]
        L = max(lens)
        x = torch.zeros(len(wavs), L)
        mask = torch.zeros(len(wavs), L, dtype=torch.long)
        for i, w in enumerate(wavs):
            x[i, :len(w)] = torch.from_numpy(w)
            mask[i, :len(w)] = 1
        t0 = time.time()
        with torch.inference_mode():
            enc = tok.encode(x, mask, return_dict=True)
        for j, c in enumerate(enc.audio_codes):
            out[f"enc/{key}/codes{j}"] = c.numpy().astype(np.int32)
            out[f"enc/{key}/sum{j}"] = np.array(float(wavs[j].astype(np.float64).sum()))
        print(f"  {fname}:enc/{key} frames {[c.shape[0] for c in enc.audio_codes]} ({time.time() - t0:.1f}s)")
    # speaker encoder
    sc = cfgm.Qwen3TTSSpeakerEncoderConfig(**cfg["speaker_encoder_config"])
    spk = mdl.Qwen3TTSSpeakerEncoder(sc).eval()
    sd = spk.state_dict()
    spk.load_state_dict({k: torch.from_numpy(synth_param("speaker_encoder." + k, v.shape, SEED)) for k, v in sd.items()})
    view = _SpeakerModelView(spk)
    for j, n in enumerate(cases["spk"]):
        w = ref_audio(n, 2000 + j)
        with torch.inference_mode():
            mel = mdl.mel_spectrogram(torch.from_numpy(w).unsqueeze(0), n_fft=1024, num_mels=128, sampling_rate=24000,
                                      hop_size=256, win_size=1024, fmin=0, fmax=12000).transpose(1, 2)
            emb = mdl.Qwen3TTSForConditionalGeneration.extract_speaker_embedding.__wrapped__(view, w, 24000) \
                if hasattr(mdl.Qwen3TTSForConditionalGeneration.extract_speaker_embedding, "__wrapped__") else \
                mdl.Qwen3TTSForConditionalGeneration.extract_speaker_embedding(view, w, 24000)
        out[f"spk/{j}/mel"] = mel[0].numpy().astype(np.float32)
        out[f"spk/{j}/emb"] = emb.numpy().astype(np.float32)
        out[f"spk/{j}/sum"] = np.array(float(w.astype(np.float64).sum()))
        print(f"  {fname}:spk/{j} mel {tuple(mel.shape)} emb {tuple(emb.shape)} |emb| {float(emb.norm()):.3f}")
    np.savez_compressed(os.path.join(HERE, fname), **out)


def make_specs():
    specs = {}
    for p in ("tiny-customvoice", "tiny-base", "1.7b-customvoice", "0.6b-customvoice", "1.7b-base", "0.6b-base"):
        m, _ = build_ref_model(p, meta=True)
        specs[p] = {k: list(v.shape) for k, v in m.state_dict().items()}
        d, _ = build_ref_codec(p, meta=True)
        specs[p + "/codec"] = {"decoder." + k: list(v.shape) for k, v in d.state_dict().items()}
        _, _, mtok, ctok = ref_shim.load_reference()
        _, ccfg = load_preset(p)
        with torch.device("meta"):
            tok = mtok.Qwen3TTSTokenizerV2Model(ctok.Qwen3TTSTokenizerV2Config(**json.loads(json.dumps(ccfg))))
        specs[p + "/encoder"] = {k: list(v.shape) for k, v in tok.state_dict().items() if k.startswith("encoder.")}
    with open(os.path.join(HERE, "param_specs.json"), "w") as f:
        json.dump(specs, f)


def make_full(only=None):
    """Production-shape fixtures (cases.full_cases): the reference's greedy generate() codes at the
    full ASSUMED dims, plus -- from the oracle, after asserting that its codes equal the reference's bit for bit --
    the top-2 margin of the processed scores at every greedy pick ([B, frames, 16], the codes' layout) and the
    hidden states of the first two and the last frame."""
    from cases import full_cases, margins_grid
    from oracle import TalkerOracle, build_prompts, generate, talker_param_specs
    from oracle.weights import synth_state_dict
    for key, case in full_cases().items():
        if only and key != only:
            continue
        t0 = time.time()
        model, cfg = build_ref_model(case["preset"])
        H = cfg["talker_config"]["hidden_size"]
        print(f"  {key}: built {case['preset']} in {time.time() - t0:.0f}s")
        t0 = time.time()
        codes, hid = run_ref_generate(model, case, case["idx"], H)
        print(f"  {key}: reference frames {[c.shape[0] for c in codes]} ({time.time() - t0:.0f}s)")
        del model
        t0 = time.time()
        o = TalkerOracle(cfg, synth_state_dict(talker_param_specs(cfg)))
        ids, ins, vcp, ref_ids = make_inputs(case, case["idx"], H)
        emb, mask, trail, pad = build_prompts(o, ids, case["languages"], case["speakers"], ins,
                                              case["non_streaming_mode"], vcp, ref_ids)
        res = generate(o, emb, mask, trail, pad, record_margins=True, **gen_kwargs(case))
        for a, b in zip(res.codes, codes):
            assert torch.equal(a, b), f"{key}: oracle codes differ from the reference at full dims"
        B = len(codes)
        mg = margins_grid(res.margins, B, res.raw_tokens.shape[1])
        print(f"  {key}: oracle == reference ({time.time() - t0:.0f}s); min margin {mg.min():.3g}, "
              f"#picks < 1e-3: {(mg < 1e-3).sum()} of {mg.size}")
        out = {"n": np.array(B), "margins": mg, "prompt_len": np.array(emb.shape[1])}
        for j, (c, h) in enumerate(zip(codes, hid)):
            out[f"codes{j}"] = c.numpy().astype(np.int32)
            out[f"hidden{j}_first"] = h[:2].numpy().astype(np.float32)
            out[f"hidden{j}_last"] = h[-1:].numpy().astype(np.float32)
        np.savez_compressed(os.path.join(HERE, f"full_{key}.npz"), **out)


class _TeacherForcer:
    """Teacher forcing inside the reference's own generate() (process-local, this script only): every call of a
    LogitsProcessorList -- the talker's (vocab V_t) once per frame and the code predictor's (vocab V_c) 15 times per
    frame, in that order (M:1671-1680, 2272) -- records the argmax of the processed scores, then returns scores that
    make the greedy argmax pick the fp32 reference's token instead, so every step sees the fp32 reference history.
    picks[b, f, g] is the reference model's own choice at frame f, codebook g (the codes' layout)."""

    def __init__(self, ref_codes, v_talker, v_cp):
        self.B, self.F = len(ref_codes), max(int(c.shape[0]) for c in ref_codes)
        self.ref = np.zeros((self.B, self.F, 16), dtype=np.int64)
        for b, c in enumerate(ref_codes):
            self.ref[b, :c.shape[0]] = c
        self.picks = np.zeros_like(self.ref)
        self.vt, self.vc = v_talker, v_cp
        self.t, self.g = 0, 0

    def __call__(self, orig, plist, input_ids, scores, **kw):
        out = orig(plist, input_ids, scores, **kw)
        V = out.shape[-1]
        if V == self.vt:
            f, col = self.t, 0
            self.t, self.g = self.t + 1, 0
        else:
            assert V == self.vc, V
            self.g += 1
            f, col = self.t - 1, self.g
        pick = out.argmax(-1).cpu().numpy()
        if f >= self.F:  # past the longest reference row (the generate's trailing step): keep the model's own choice
            return out
        self.picks[:, f, col] = pick
        forced = torch.as_tensor(self.ref[:, f, col], device=out.device)
        hard = torch.full_like(out, float("-inf"))
        hard.scatter_(1, forced[:, None], 0.0)
        return hard


def make_full_bf16(only=None):
    """The reference itself in bf16 (the examples' dtype, examples/test_model_12hz_custom_voice.py:30: parameters cast to
    bf16 as from_pretrained(dtype=torch.bfloat16) loads them; buffers such as RoPE inv_freq stay fp32), eager CPU, on
    the full-dim cases cv17_b8_stream, cv06_b1_nonstream and cv17_b2_long (256 frames): (1) teacher-forced on the fp32 reference codes of
    full_<key>.npz -- its own greedy pick at every position; (2) free-running greedy codes.  Written to
    full_<key>_refbf16.npz: the calibration of bf16 agreement (tests/test_gpu_full.py)."""
    import transformers.generation.logits_process as lp
    from cases import full_cases
    for key in ("cv17_b8_stream", "cv06_b1_nonstream", "cv17_b2_long", "cv17_b2_longctx", "cv17_b2_longctx4"):
        if only and key != only:
            continue
        case = full_cases()[key]
        t0 = time.time()
        model, cfg = build_ref_model(case["preset"])
        for p in model.parameters():
            p.data = p.data.to(torch.bfloat16)
        H = cfg["talker_config"]["hidden_size"]
        z = np.load(os.path.join(HERE, f"full_{key}.npz"))
        ref = [z[f"codes{j}"] for j in range(int(z["n"]))]
        tf = _TeacherForcer(ref, cfg["talker_config"]["vocab_size"],
                            cfg["talker_config"]["code_predictor_config"]["vocab_size"])
        orig = lp.LogitsProcessorList.__call__
        lp.LogitsProcessorList.__call__ = lambda self, ids, sc, **kw: tf(orig, self, ids, sc, **kw)
        try:
            tcase = dict(case, max_new_tokens=tf.F + 1)
            run_ref_generate(model, tcase, case["idx"], H)
        finally:
            lp.LogitsProcessorList.__call__ = orig
        agree = np.mean([np.mean(tf.picks[b, :r.shape[0]] == r) for b, r in enumerate(ref)])
        print(f"  {key}: reference bf16 teacher-forced agreement with its fp32 codes {agree:.4%} "
              f"({time.time() - t0:.0f}s)")
        t0 = time.time()
        codes, _ = run_ref_generate(model, case, case["idx"], H)
        print(f"  {key}: reference bf16 free-running frames {[c.shape[0] for c in codes]} ({time.time() - t0:.0f}s)")
        out = {"n": np.array(len(ref)), "picks_tf": tf.picks.astype(np.int32)}
        for j, c in enumerate(codes):
            out[f"codes_free{j}"] = c.numpy().astype(np.int32)
        np.savez_compressed(os.path.join(HERE, f"full_{key}_refbf16.npz"), **out)
        del model


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--full", action="store_true")
    ap.add_argument("--only", default=None)
    a = ap.parse_args()
    torch.set_num_threads(8)
    if a.only in (None, "specs"):
        make_specs()
    if a.only in (None, "talker"):
        make_tiny_talker()
    if a.only in (None, "codec"):
        make_codec("tiny-customvoice", {"single": [40], "batch_ragged": [23, 9], "chunked": [330]},
                   "codec_tiny.npz")
        make_codec("1.7b-customvoice", {"single": [38], "batch_ragged": [12, 5]}, "codec_full.npz")
    if a.only in (None, "frontend"):
        make_frontend("tiny-base", "tiny", "frontend_tiny.npz")
        make_frontend("1.7b-base", "full", "frontend_full.npz")
    if a.only in (None, "codec_chunks"):
        # full-dim chunk restarts (K:885-895): 300 frames = one chunk, 325 / 700 = restarts with 25 frames of left
        # context, and a ragged pair whose long row restarts while the short one is zero padding
        make_codec("1.7b-customvoice", {"t300": [300], "t325": [325], "t700": [700], "ragged_325_40": [325, 40]},
                   "codec_full_chunks.npz", stride=17)
    if a.full or ((a.only or "").startswith("full") and not (a.only or "").startswith("full_bf16")):
        make_full(a.only.split(":", 1)[1] if a.only and ":" in a.only else None)
    if a.full or (a.only or "").startswith("full_bf16"):
        make_full_bf16(a.only.split(":", 1)[1] if a.only and ":" in a.only else None)


if __name__ == "__main__":
    main()
