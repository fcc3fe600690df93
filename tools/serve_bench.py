"""Continuous batching vs padded one-shot batches on BASELINE.json configs[3]'s per-GPU work.

configs[3] = Qwen3-TTS-12Hz-1.7B VoiceDesign, 64 mixed-length requests data-parallel over 8 GPUs (SURVEY §8d:
text ~ U[40, 300] tokens, instruct ~ U[10, 60] tokens, F ~ U[64, 320] frames; non_streaming_mode=True, the
voice-design wrapper's default; sampling with the wrapper defaults).  Per request the frame count is fixed
(ignore_eos + a per-request cap), so both schedules generate the same audio:

* padded: the reference's schedule -- the requests in batches of `--slots`, each batch decoded until its longest
  request ends (finished rows emit EOS padding), M:2272-2292;
* serve: TalkerEngine.serve through `--slots` batch rows, a row refilled as soon as its request ends.

Both include prompt assembly and the codec decode of every request.  Prints one JSON line per schedule.

    python tools/serve_bench.py [--requests 8] [--slots 8] [--extra-slots 16,32]
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
sys.path.insert(0, os.path.join(REPO, "qwen3-tts_amd"))
sys.path.insert(0, REPO)

from bench import make_weights  # noqa: E402


def workload(n, seed=4):
    g = np.random.default_rng([seed, 99])
    reqs = []
    for i in range(n):
        t, k, f = int(g.integers(40, 301)), int(g.integers(10, 61)), int(g.integers(64, 321))
        body = g.integers(1000, 150000, t).tolist()
        ids = torch.tensor([[151644, 77091, 198] + body + [151645, 198, 151644, 77091, 198]], dtype=torch.long)
        ins = torch.tensor([[151644, 872, 198] + g.integers(1000, 150000, k).tolist() + [151645, 198]],
                           dtype=torch.long)
        reqs.append((ids, ins, f))
    return reqs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="1.7b-voicedesign")
    ap.add_argument("--requests", type=int, default=8)
    ap.add_argument("--slots", type=int, default=8)
    ap.add_argument("--extra-slots", default="")
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    from qwen_tts import Qwen3TTSModel
    from qwen_tts.talker import GenParams
    _, W, CW = make_weights(a.preset, dev, 1, 0)
    tts = Qwen3TTSModel.from_pretrained(f"synthetic:{a.preset}", device_map=str(dev), dtype=torch.bfloat16,
                                        weights=W, codec_weights=CW)
    del W, CW
    m, eng = tts.model, tts.model.engine
    reqs = workload(a.requests)
    F = [f for _, _, f in reqs]
    audio_s = 0.08 * sum(F)
    # F = max_new_tokens - 1 frames, as in bench.py; every row runs with ignore_eos so its length is exact
    gen = dict(do_sample=True, top_k=50, top_p=1.0, temperature=0.9, subtalker_dosample=True, subtalker_top_k=50,
               subtalker_top_p=1.0, subtalker_temperature=0.9, repetition_penalty=1.05, ignore_eos=True)

    def prompts(sel):
        return m.build_prompts([reqs[i][0] for i in sel], ["english"] * len(sel), None, [reqs[i][1] for i in sel],
                               True)

    def padded(slots, seed):
        codes = [None] * len(reqs)
        for b0 in range(0, len(reqs), slots):
            sel = list(range(b0, min(b0 + slots, len(reqs))))
            emb, mask, trail, pad = prompts(sel)
            gp = GenParams(max_new_tokens=max(F[i] for i in sel) + 1, seed=seed, **gen)
            out, _ = eng.generate_from_embeds(emb, mask, trail, pad, gp)
            for j, i in enumerate(sel):
                codes[i] = out[j][:F[i]]
        return codes

    def serve(slots, seed):
        emb, mask, trail, pad = prompts(list(range(len(reqs))))
        P = emb.shape[1]
        n_real = mask.sum(-1).tolist()
        rq = [(emb[i, P - int(n_real[i]):], trail[i], F[i]) for i in range(len(reqs))]
        gp = GenParams(max_new_tokens=max(F) + 1, seed=seed, **gen)
        codes = [None] * len(reqs)
        for i, c, _ in eng.serve(rq, pad, gp, slots=slots):
            codes[i] = c
        return codes

    def run(fn, slots):
        fn(slots, 1)  # warmup (graph capture, sessions)
        ts = []
        for r in range(a.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            codes = fn(slots, 10 + r)
            assert [c.shape[0] for c in codes] == F, [c.shape[0] for c in codes]
            wavs, sr = m.speech_tokenizer.decode([{"audio_codes": c} for c in codes])
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts))

    slot_list = [a.slots] + [int(x) for x in a.extra_slots.split(",") if x]
    for name, fn in (("padded", padded), ("serve", serve)):
        for slots in slot_list:
            if name == "padded" and slots != a.slots:
                continue
            dt = run(fn, slots)
            st = getattr(eng, "serve_stats", {}) if name == "serve" else {}
            print(json.dumps({"schedule": name, "slots": slots, "requests": a.requests, "frames": F,
                              "frames_replayed": st.get("frames"), "frames_min": -(-sum(F) // slots),
                              "audio_s": round(audio_s, 2), "wall_s": round(dt, 4),
                              "audio_s_per_s": round(audio_s / dt, 2),
                              "workload": f"{a.preset} configs[3] shard, text U[40,300], instruct U[10,60], "
                                          "F U[64,320], sampling, ignore_eos + per-request cap, + codec decode"}),
                  flush=True)


if __name__ == "__main__":
    main()
