"""Where the first packet's time goes at the bench configuration (1.7B synthetic, B=8 and B=1, 200-token prompts,
streaming text): prompt assembly, prefill + first frame (generate with max_new_tokens=1), each further frame, and
the codec's first incremental feed (first_chunk_frames = 2 frames)."""
import os
import sys
import time
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "qwen3-tts_amd"))
import bench  # noqa: E402


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    return float(np.median(ts))


def main():
    dev = torch.device("cuda:0")
    from qwen_tts import Qwen3TTSModel
    cfg, W, CW = bench.make_weights("1.7b-customvoice", dev, 1, 0)
    tts = Qwen3TTSModel.from_pretrained("synthetic:1.7b-customvoice", device_map=str(dev), dtype=torch.bfloat16,
                                        weights=W, codec_weights=CW)
    m = tts.model
    spk = ["vivian", "ryan", "serena", "aiden", "eric", "dylan", "sohee", "ono_anna"]
    gen = dict(do_sample=True, top_k=50, top_p=1.0, temperature=0.9, subtalker_dosample=True, subtalker_top_k=50,
               subtalker_top_p=1.0, subtalker_temperature=0.9, repetition_penalty=1.05, ignore_eos=True)
    for B in (8, 1):
        ids = [bench.synth_ids(200, i) for i in range(B)]
        kw = dict(input_ids=ids, languages=["english"] * B, speakers=spk[:B], non_streaming_mode=False, seed=7)
        t_prompt = timed(lambda: m.build_prompts(ids, ["english"] * B, spk[:B], None, False, None, None))
        t1 = timed(lambda: m.generate(max_new_tokens=1, **kw, **gen))
        t6 = timed(lambda: m.generate(max_new_tokens=6, **kw, **gen))
        codes = torch.randint(1, 2048, (B, 2, 16), device=dev, dtype=torch.int32)
        dec = m.speech_tokenizer.model

        def feed():
            dec.stream(B, 325).feed(codes)
        t_codec = timed(feed)

        def first():
            for _ in m.stream(**kw, max_new_tokens=257, **gen):
                break
        t_fp = timed(first)
        print(f"B={B}: prompt assembly {t_prompt:.1f} ms | generate(1 frame) {t1:.1f} | generate(6) {t6:.1f} "
              f"(+{(t6 - t1) / 5:.2f} per frame) | codec feed of 2 frames {t_codec:.1f} | stream first packet {t_fp:.1f}",
              flush=True)


if __name__ == "__main__":
    main()
