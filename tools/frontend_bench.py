"""Voice-clone front-end latency on one MI355X (3 s reference clips at 24 kHz).

    python tools/frontend_bench.py [--preset 1.7b-base] [--dtype bf16] [--batch 1 4] [--reps 20] [--cpu]

Times (HIP events around the whole call, inputs already on the device):
  * Qwen3TTSTokenizer encode (12 Hz Mimi encoder -> 16 codebooks) of B clips,
  * extract_speaker_embedding (mel + ECAPA) of one clip,
and, with --cpu, the fp32 CPU oracle of the same work (oracle/encoder.py, oracle/speaker.py; measurement only).
Synthetic weights (device RNG) at the preset's dims.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "qwen3-tts_amd"), os.path.join(REPO, "tests", "golden")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="1.7b-base")
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--batch", type=int, nargs="+", default=[1, 4])
    ap.add_argument("--samples", type=int, default=72000)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--cpu", action="store_true")
    a = ap.parse_args()
    from cases import ref_audio
    from qwen_tts.encoder import TokenizerEncoder, encoder_specs
    from qwen_tts.speaker import SpeakerEncoder, speaker_specs
    from qwen_tts.weights import PRESETS, read_json, synthetic
    dev = torch.device("cuda:0")
    d = os.path.join(PRESETS, a.preset)
    cfg, ccfg = read_json(os.path.join(d, "config.json")), read_json(os.path.join(d, "speech_tokenizer", "config.json"))
    enc = TokenizerEncoder(ccfg, synthetic(encoder_specs(ccfg), dev), dtype=a.dtype, device=dev)
    spk = SpeakerEncoder(cfg, synthetic(speaker_specs(cfg), dev), dtype=a.dtype, device=dev)
    out = {"preset": a.preset, "dtype": a.dtype, "samples": a.samples}

    def timed(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ts = []
        for _ in range(a.reps):
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        return float(np.median(ts))

    wav = torch.from_numpy(ref_audio(a.samples, 7)).to(dev)
    for B in a.batch:
        wavs = [wav] * B
        out[f"encode_ms_b{B}"] = timed(lambda: enc.encode(wavs))
    out["speaker_ms"] = timed(lambda: spk.embed(wav))
    out["mel_ms"] = timed(lambda: spk.mel(wav))
    if a.cpu:
        from oracle import synth_param
        from oracle.encoder import EncoderOracle, encoder_param_specs
        from oracle.speaker import SpeakerOracle, speaker_param_specs
        torch.set_num_threads(min(16, os.cpu_count() or 1))
        eo = EncoderOracle(ccfg, {n: synth_param(n, s) for n, s in encoder_param_specs(ccfg)})
        so = SpeakerOracle(cfg, {n: synth_param(n, s) for n, s in speaker_param_specs(cfg)})
        w = ref_audio(a.samples, 7)
        t0 = time.perf_counter()
        eo.encode([w])
        out["cpu_encode_ms_b1"] = 1e3 * (time.perf_counter() - t0)
        t0 = time.perf_counter()
        so.embed(w)
        out["cpu_speaker_ms"] = 1e3 * (time.perf_counter() - t0)
        out["cpu_threads"] = torch.get_num_threads()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
