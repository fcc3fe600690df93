"""Code-predictor logits at the bench configuration (1.7B synthetic weights, B=8): spread, and how the sampler's
value-histogram top-k path (bins of 1/16 below the row max, boundary bin ranked by one wave when it holds <= 64
keys) would see them.  Reads the last step's logits buffer of every CP lane after a short generate()."""
import os
import sys
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
    ids = [bench.synth_ids(200, i) for i in range(8)]
    gen = dict(max_new_tokens=9, do_sample=True, top_k=50, top_p=1.0, temperature=0.9, subtalker_dosample=True,
               subtalker_top_k=50, subtalker_top_p=1.0, subtalker_temperature=0.9, repetition_penalty=1.05,
               ignore_eos=True)
    tts.model.generate(input_ids=ids, languages=["english"] * 8, speakers=["vivian"] * 8, non_streaming_mode=False,
                       seed=1, **gen)
    torch.cuda.synchronize()
    for s in tts.model.engine.all_sessions():
        for ln in [s.cp]:
            lg = ln.logits.float().cpu().numpy()[: ln.nb] / 0.9
            for r, row in enumerate(lg):
                m = row.max()
                srt = np.sort(row)[::-1]
                bins = np.floor((m - row) * 16).astype(int)
                kb = int(np.floor((m - srt[49]) * 16))
                print(f"row {r}: std {row.std():.3f} max-kth {m - srt[49]:.3f} boundary bin {kb} holds "
                      f"{int((bins == kb).sum())} keys, above {int((bins < kb).sum())}")


if __name__ == "__main__":
    main()
