"""Cross-check of bench.py's CPU baseline (the oracle, `cpu_baseline.kind = "port"`) against the reference itself
(the CPU baseline stand-in must be within 10 % of the shimmed reference on the same workload).

Container only (imports /root/reference through ref_shim, like make_golden.py; nothing on the GPU box runs it).
Workload: BASELINE.json configs[2] shape -- Qwen3-TTS-12Hz-1.7B CustomVoice, B=8 x 200-token synthetic prompts,
streaming text, --frames frames (greedy: the reference's generate() has no ignore_eos, and greedy on these seeded
weights runs every row to the frame cap), then the 12 Hz codec decode of all 8 rows to PCM; the same seeded weights
and token ids for both, torch.set_num_threads(--threads), each path timed once after a 2-frame warm-up.
Writes the two rates (audio-seconds / second) and their ratio to --out (JSON).

    python tests/golden/cpu_baseline_xval.py --threads 8 --frames 24 --out profiles/r05_cpu_baseline_xval.json
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [HERE, REPO]

from cases import FULL_SPEAKERS, text_ids  # noqa: E402
import make_golden as mg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--frames", type=int, default=24)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--prompt", type=int, default=200)
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "r05_cpu_baseline_xval.json"))
    a = ap.parse_args()
    torch.set_num_threads(a.threads)
    preset = "1.7b-customvoice"
    B = a.batch
    ids = [text_ids(a.prompt, 7000 + j) for j in range(B)]
    langs, spk = ["english"] * B, (FULL_SPEAKERS * 2)[:B]
    gen = dict(do_sample=False, subtalker_dosample=False, top_k=50, top_p=1.0, temperature=0.9, subtalker_top_k=50,
               subtalker_top_p=1.0, subtalker_temperature=0.9, repetition_penalty=1.05)

    # ---- the reference (shimmed transformers 5.x -> 4.57 behaviour, make_golden.py)
    model, cfg = mg.build_ref_model(preset)
    dec, ccfg = mg.build_ref_codec(preset)

    def ref_run(frames):
        t0 = time.perf_counter()
        with torch.no_grad():
            codes, _ = model.generate(input_ids=ids, languages=langs, speakers=spk, non_streaming_mode=False,
                                      max_new_tokens=frames + 1, **gen)
        wavs = mg.ref_codec_decode(dec, ccfg, [c.numpy() for c in codes])
        return sum(w.shape[0] for w in wavs) / 24000.0, time.perf_counter() - t0, [c.shape[0] for c in codes]
    ref_run(2)
    r_audio, r_dt, r_frames = ref_run(a.frames)
    del model, dec

    # ---- the oracle (bench.py's cpu_baseline path: build_prompts + generate + CodecOracle.decode)
    from oracle import CodecOracle, TalkerOracle, build_prompts, codec_param_specs, generate, load_preset
    from oracle.talker import talker_param_specs
    from oracle.weights import synth_state_dict
    cfg, ccfg = load_preset(preset)
    o = TalkerOracle(cfg, synth_state_dict(talker_param_specs(cfg)))
    co = CodecOracle(ccfg, synth_state_dict(codec_param_specs(ccfg)))

    def oracle_run(frames):
        t0 = time.perf_counter()
        with torch.no_grad():
            emb, mask, trail, pad = build_prompts(o, ids, langs, spk, None, False)
            res = generate(o, emb, mask, trail, pad, max_new_tokens=frames + 1, **gen)
            wav = co.decode(torch.stack(res.codes))
        return sum(w.shape[0] for w in wav) / 24000.0, time.perf_counter() - t0, [c.shape[0] for c in res.codes]
    oracle_run(2)
    o_audio, o_dt, o_frames = oracle_run(a.frames)

    rr, orr = r_audio / r_dt, o_audio / o_dt
    out = {"workload": f"Qwen3-TTS-12Hz-1.7B CustomVoice, B={B} x {a.prompt}-token prompts, streaming text, "
                       f"{a.frames} greedy frames + codec decode (seeded synthetic weights, same ids)",
           "threads": a.threads, "host_cpu_count": os.cpu_count(),
           "reference": {"audio_seconds": r_audio, "wall_s": r_dt, "audio_s_per_s": rr, "frames": r_frames},
           "oracle": {"audio_seconds": o_audio, "wall_s": o_dt, "audio_s_per_s": orr, "frames": o_frames},
           "oracle_over_reference": orr / rr,
           "within_10pct": abs(orr / rr - 1.0) <= 0.10}
    print(json.dumps(out, indent=1))
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
