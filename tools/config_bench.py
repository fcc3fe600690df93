"""BASELINE.json's other configurations, measured per GPU on one MI355X (bench.py measures configs[2]).

configs[1]: Qwen3-TTS-12Hz-0.6B CustomVoice, one utterance of ~120 text tokens, greedy (do_sample and
            subtalker_dosample off), batch 1; non_streaming_mode=True (the custom-voice wrapper's default),
            128 frames (ignore_eos).  Reports the end-to-end latency (prompt + AR + codec), audio-s/s (= RTF at
            batch 1) and the stream() first packet.
configs[4]: Qwen3-TTS-12Hz-1.7B-Base voice clone, batch 32 over 8 GPUs = 4 requests per GPU: a 3 s 24 kHz
            reference clip per request (ICL mode, 40-token reference text) -> tokenizer encode + x-vector, AR decode of
            256 frames (sampling, wrapper defaults, streaming text -- the voice-clone wrapper's default), codec decode
            of cat(ref codes, codes) and the reference cut (generate_voice_clone).  Reports whole-job audio-s/s per GPU
            and the first-packet p50 of stream_voice_clone's path (request submit, reference encode included -> first
            PCM chunk).

Weights are seeded synthetic at the presets' dims; token ids are synthetic (no BPE offline).  One JSON line per
configuration.

    python tools/config_bench.py [--configs 1 4] [--reps 3]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "qwen3-tts_amd"), os.path.join(REPO, "tests", "golden")]

from bench import synth_ids  # noqa: E402


def timed(fn, reps):
    fn()
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)), out


def config1(reps):
    from qwen_tts import Qwen3TTSModel
    tts = Qwen3TTSModel.from_pretrained("synthetic:0.6b-customvoice", dtype=torch.bfloat16)
    m = tts.model
    ids = [synth_ids(120, 0)]
    F = 128
    kw = dict(input_ids=ids, languages=["english"], speakers=["vivian"], non_streaming_mode=True,
              max_new_tokens=F + 1, do_sample=False, subtalker_dosample=False, repetition_penalty=1.05,
              ignore_eos=True)

    def one():
        codes, _ = m.generate(**kw)
        wavs, sr = m.speech_tokenizer.decode([{"audio_codes": c} for c in codes])
        return sum(w.shape[0] for w in wavs) / sr

    dt, audio = timed(one, reps)

    def first():
        for _ in m.stream(**kw):
            break

    fp, _ = timed(first, reps)
    return {"config": "configs[1] 0.6B CustomVoice B=1 greedy, 120-token text, non-streaming prompt, 128 frames + codec",
            "latency_ms": round(1e3 * dt, 1), "audio_s": round(audio, 3), "audio_s_per_s": round(audio / dt, 2),
            "rtf": round(audio / dt, 2), "first_packet_p50_ms": round(1e3 * fp, 1)}


def config4(reps, B=4):
    from cases import ref_audio, ref_text_ids
    from qwen_tts import Qwen3TTSModel
    tts = Qwen3TTSModel.from_pretrained("synthetic:1.7b-base", dtype=torch.bfloat16)
    m = tts.model
    clips = [(ref_audio(72000, 100 + i), 24000) for i in range(B)]
    ids = [synth_ids(120, 50 + i) for i in range(B)]
    ref_ids = [ref_text_ids(40, 60 + i) for i in range(B)]
    F = 256
    gen = dict(max_new_tokens=F + 1, do_sample=True, top_k=50, top_p=1.0, temperature=0.9, subtalker_dosample=True,
               subtalker_top_k=50, subtalker_top_p=1.0, subtalker_temperature=0.9, repetition_penalty=1.05,
               ignore_eos=True)

    def prompt():
        # generate_voice_clone's front end (W:356-458) on token ids: encode + x-vector of every reference clip
        items = tts.create_voice_clone_prompt(ref_audio=clips, ref_text=["ref"] * B)
        return tts._prompt_items_to_voice_clone_prompt(items)

    def one():
        vcp = prompt()
        codes, _ = m.generate(input_ids=ids, ref_ids=ref_ids, voice_clone_prompt=vcp, languages=["english"] * B,
                              non_streaming_mode=False, **gen)
        refs = vcp["ref_code"]
        dec = [torch.cat([refs[i].cpu().long(), c], 0) for i, c in enumerate(codes)]
        wavs, sr = m.speech_tokenizer.decode([{"audio_codes": c} for c in dec])
        out = [w[int(int(refs[i].shape[0]) / dec[i].shape[0] * w.shape[0]):] for i, w in enumerate(wavs)]
        return sum(w.shape[0] for w in out) / sr, int(refs[0].shape[0])

    dt, (audio, R) = timed(one, reps)

    def first():
        vcp = prompt()
        for _ in m.stream(input_ids=ids, ref_ids=ref_ids, voice_clone_prompt=vcp, languages=["english"] * B,
                          non_streaming_mode=False, **gen):
            break

    fp, _ = timed(first, reps)
    enc, _ = timed(prompt, reps)
    # first-packet breakdown: prompt assembly (ICL layout), prefill + first frame, codec decode of the reference
    # frames + one generated frame
    vcp = prompt()
    asm, _ = timed(lambda: m.build_prompts(ids, ["english"] * B, None, None, False, vcp, ref_ids), reps)
    g1, _ = timed(lambda: m.generate(input_ids=ids, ref_ids=ref_ids, voice_clone_prompt=vcp, languages=["english"] * B,
                                     non_streaming_mode=False, **dict(gen, max_new_tokens=2)), reps)
    dec = m.speech_tokenizer.model
    cc = torch.randint(1, 2048, (B, R + 1, 16), device="cuda", dtype=torch.int32)
    cf, _ = timed(lambda: dec.stream(B, 325).feed(cc), reps)
    return {"config": f"configs[4] 1.7B-Base voice clone, {B} requests per GPU (32 over 8 GPUs): 3 s reference clips "
                      f"({R} ref frames, ICL) encode + x-vector, 120-token text, {F} frames sampled + codec",
            "latency_ms": round(1e3 * dt, 1), "audio_s": round(audio, 3), "audio_s_per_s": round(audio / dt, 2),
            "rtf_per_utterance": round(audio / dt / B, 2), "first_packet_p50_ms": round(1e3 * fp, 1),
            "voice_clone_prompt_ms": round(1e3 * enc, 2), "prompt_assembly_ms": round(1e3 * asm, 2),
            "generate_1_frame_ms": round(1e3 * g1, 2), "codec_ref_plus_1_frame_ms": round(1e3 * cf, 2)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", type=int, nargs="+", default=[1, 4])
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    for c in a.configs:
        out = config1(a.reps) if c == 1 else config4(a.reps)
        print(json.dumps(out), flush=True)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
