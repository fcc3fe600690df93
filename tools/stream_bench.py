"""stream() at the bench configuration (1.7B synthetic weights, B=8 x 200-token prompts, streaming text, 256 frames,
sampling): first-packet latency and whole-stream wall time, stateful incremental codec (default) vs the stateless
window re-decode (left_context=325, the reference-exact form of round 1)."""
import os
import sys
import time
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "qwen3-tts_amd"))
import bench  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    from qwen_tts import Qwen3TTSModel
    cfg, W, CW = bench.make_weights("1.7b-customvoice", dev, 1, 0)
    tts = Qwen3TTSModel.from_pretrained("synthetic:1.7b-customvoice", device_map=str(dev), dtype=torch.bfloat16,
                                        weights=W, codec_weights=CW)
    B, F = 8, 256
    ids = [bench.synth_ids(200, i) for i in range(B)]
    spk = ["vivian", "ryan", "serena", "aiden", "eric", "dylan", "sohee", "ono_anna"]
    gen = dict(max_new_tokens=F + 1, do_sample=True, top_k=50, top_p=1.0, temperature=0.9, subtalker_dosample=True,
               subtalker_top_k=50, subtalker_top_p=1.0, subtalker_temperature=0.9, repetition_penalty=1.05,
               ignore_eos=True)

    def run(ctx):
        t0 = time.perf_counter()
        first, n = None, 0
        for b, pcm, last in tts.model.stream(input_ids=ids, languages=["english"] * B, speakers=spk,
                                             non_streaming_mode=False, seed=7, left_context=ctx, **gen):
            if first is None:
                torch.cuda.synchronize()
                first = time.perf_counter() - t0
            n += pcm.numel()
        torch.cuda.synchronize()
        return first * 1e3, (time.perf_counter() - t0) * 1e3, n

    for ctx in (None, 325):
        run(ctx)
        r = [run(ctx) for _ in range(3)]
        fp = float(np.median([x[0] for x in r]))
        tot = float(np.median([x[1] for x in r]))
        print(f"left_context={ctx}: first packet p50 {fp:.1f} ms, whole stream {tot:.1f} ms, "
              f"{r[0][2] / 24000 / (tot / 1e3):.1f} audio-s/s", flush=True)
    t0 = time.perf_counter()
    codes, _ = tts.model.generate(input_ids=ids, languages=["english"] * B, speakers=spk, non_streaming_mode=False,
                                  seed=7, **gen)
    tts.model.speech_tokenizer.decode([{"audio_codes": c} for c in codes])
    torch.cuda.synchronize()
    print(f"one-shot generate + decode: {(time.perf_counter() - t0) * 1e3:.1f} ms", flush=True)


if __name__ == "__main__":
    main()
