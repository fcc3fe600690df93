"""A short configs[2]-shaped decode for rocprofv3 --kernel-trace: 1.7B CustomVoice, B=8 x 200-token prompts, two
warm-up generates, then one of 24 frames; tools/frame_trace_reduce.py turns the trace into one frame's kernel sequence
(durations and the gaps between dependent launches)."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "qwen3-tts_amd")]
from bench import make_weights, synth_ids  # noqa: E402
from qwen_tts import Qwen3TTSModel  # noqa: E402

dev = torch.device("cuda:0")
cfg, W, CW = make_weights("1.7b-customvoice", dev, 1, 0)
tts = Qwen3TTSModel.from_pretrained("synthetic:1.7b-customvoice", device_map="cuda:0", dtype=torch.bfloat16, weights=W,
                                    codec_weights=CW)
B = int(os.environ.get("QT_FT_B", "8"))
ids = [synth_ids(200, i) for i in range(B)]
spk = (["vivian", "ryan", "serena", "aiden", "eric", "dylan", "sohee", "ono_anna"] * 2)[:B]
gen = dict(do_sample=True, top_k=50, top_p=1.0, temperature=0.9, subtalker_dosample=True, subtalker_top_k=50,
           subtalker_top_p=1.0, subtalker_temperature=0.9, repetition_penalty=1.05, ignore_eos=True)
for n in (25, 25, 25):
    tts.model.generate(input_ids=ids, languages=["english"] * B, speakers=spk, non_streaming_mode=False, seed=1,
                       max_new_tokens=n, **gen)
torch.cuda.synchronize()
print("done")
