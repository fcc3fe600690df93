"""Pin the oracle (CPU fp32 restatement) to golden vectors produced by the reference itself.

The fixtures come from tests/golden/make_golden.py, which imports /root/reference/qwen_tts (shimmed,
SURVEY.md §8c) and runs `Qwen3TTSForConditionalGeneration.generate` / `Qwen3TTSTokenizerV2Model.decode`
on the same seeded synthetic weights.  CPU only.
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle import (CodecOracle, TalkerOracle, build_prompts, codec_param_specs, generate, load_preset,
                    synth_state_dict, talker_param_specs, tokenizer_decode)
from cases import gen_kwargs, make_inputs, talker_cases

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def tiny_talkers():
    out = {}
    for p in ("tiny-customvoice", "tiny-voicedesign"):
        cfg, _ = load_preset(p)
        out[p] = (cfg, synth_state_dict(talker_param_specs(cfg)))
    return out


def test_param_specs_match_reference():
    specs = json.load(open(os.path.join(GOLD, "param_specs.json")))
    for p in ("tiny-customvoice", "1.7b-customvoice", "0.6b-customvoice", "0.6b-base"):
        cfg, ccfg = load_preset(p)
        ref = {k: v for k, v in specs[p].items() if not k.startswith("speaker_encoder")}
        assert {k: list(v) for k, v in talker_param_specs(cfg)} == ref
        assert {k: list(v) for k, v in codec_param_specs(ccfg)} == specs[p + "/codec"]


def run_oracle_case(cfg, W, key, case, idx, **over):
    o = TalkerOracle(cfg, W)
    H = cfg["talker_config"]["hidden_size"]
    ids, ins, vcp, ref_ids = make_inputs(case, idx, H)
    emb, mask, trail, pad = build_prompts(o, ids, case["languages"], case["speakers"], ins,
                                          case["non_streaming_mode"], vcp, ref_ids)
    kw = gen_kwargs(case)
    kw.update(over)
    return generate(o, emb, mask, trail, pad, seed=case.get("seed", 0), **kw)


@pytest.mark.parametrize("key", list(talker_cases()))
def test_oracle_generate_matches_reference(tiny_talkers, key):
    z = np.load(os.path.join(GOLD, "tiny_talker.npz"))
    cases = talker_cases()
    case = cases[key]
    preset = "tiny-voicedesign" if key.startswith("vd_") else "tiny-customvoice"
    cfg, W = tiny_talkers[preset]
    res = run_oracle_case(cfg, W, key, case, list(cases).index(key))
    assert len(res.codes) == int(z[f"{key}/n"])
    for j, c in enumerate(res.codes):
        np.testing.assert_array_equal(c.numpy(), z[f"{key}/codes{j}"])
        np.testing.assert_allclose(res.hidden[j].numpy(), z[f"{key}/hidden{j}"], rtol=1e-4, atol=1e-5)


def test_oracle_eos_ragged_matches_reference(tiny_talkers):
    z = np.load(os.path.join(GOLD, "tiny_talker.npz"))
    cfg, W = tiny_talkers["tiny-customvoice"]
    W = dict(W)
    eos = cfg["talker_config"]["codec_eos_token_id"]
    head = W["talker.codec_head.weight"].copy()
    head[eos] = head[int(z["eos_b2/donor"])]
    W["talker.codec_head.weight"] = head
    cases = talker_cases()
    key = "cv_b2_stream_dialect"
    res = run_oracle_case(cfg, W, key, dict(cases[key], max_new_tokens=24), list(cases).index(key))
    lens = [c.shape[0] for c in res.codes]
    assert lens[0] != lens[1], "fixture is meant to stop the two rows at different frames"
    for j, c in enumerate(res.codes):
        np.testing.assert_array_equal(c.numpy(), z[f"eos_b2/codes{j}"])


@pytest.mark.parametrize("fname,preset", [("codec_tiny.npz", "tiny-customvoice"), ("codec_full.npz", "1.7b-customvoice"),
                                           ("codec_full_chunks.npz", "1.7b-customvoice")])
def test_oracle_codec_matches_reference(fname, preset):
    z = np.load(os.path.join(GOLD, fname))
    _, ccfg = load_preset(preset)
    o = CodecOracle(ccfg, synth_state_dict(codec_param_specs(ccfg)))
    keys = sorted({k.split("/")[0] for k in z.files})
    for key in keys:
        n = len([k for k in z.files if k.startswith(key + "/codes")])
        codes = [z[f"{key}/codes{j}"].astype(np.int64) for j in range(n)]
        wavs = tokenizer_decode(o, codes)
        for j, w in enumerate(wavs):
            assert w.shape[0] == int(z[f"{key}/len{j}"])
            if f"{key}/wav{j}" in z.files:
                np.testing.assert_allclose(w, z[f"{key}/wav{j}"], atol=2e-5, rtol=0)
            else:
                stride = int(z[f"{key}/stride"]) if f"{key}/stride" in z.files else 7
                np.testing.assert_allclose(w[::stride], z[f"{key}/wav{j}_stride"], atol=2e-5, rtol=0)
                s = z[f"{key}/wav{j}_sum"]
                np.testing.assert_allclose([w.astype(np.float64).sum(), (w.astype(np.float64) ** 2).sum()], s,
                                           rtol=1e-4)


@pytest.mark.parametrize("key", ["cv06_b1_nonstream"] + (["cv17_b8_stream", "vd17_b4_instruct", "base17_b2_clone"]
                                           if os.environ.get("QT_SLOW") else []))
def test_oracle_full_dims_matches_reference(key):
    """Full ASSUMED dims (configs[1] shape; configs[2] with QT_SLOW=1, ~4 min): the oracle's greedy codes equal the
    reference's (tests/golden/full_<key>.npz) and its recorded top-2 margins are the fixture's."""
    from cases import full_cases, make_inputs, margins_grid
    case = full_cases()[key]
    cfg, _ = load_preset(case["preset"])
    z = np.load(os.path.join(GOLD, f"full_{key}.npz"))
    o = TalkerOracle(cfg, synth_state_dict(talker_param_specs(cfg), threads=8))
    ids, ins, vcp, ref_ids = make_inputs(case, case["idx"], cfg["talker_config"]["hidden_size"])
    emb, mask, trail, pad = build_prompts(o, ids, case["languages"], case["speakers"], ins, case["non_streaming_mode"],
                                          vcp, ref_ids)
    with torch.no_grad():
        res = generate(o, emb, mask, trail, pad, record_margins=True, **gen_kwargs(case))
    for j, c in enumerate(res.codes):
        np.testing.assert_array_equal(c.numpy(), z[f"codes{j}"])
    np.testing.assert_allclose(margins_grid(res.margins, len(res.codes), res.raw_tokens.shape[1]), z["margins"],
                               rtol=1e-5, atol=1e-7)
