"""Codec decode time (12 Hz decoder, 1.7B preset dims, seeded synthetic weights): B utterances x T frames.
    python tools/codec_bench.py [B] [T]        (QT_NO_IGEMM=1 selects the untiled GEMM for A/B)"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "qwen3-tts_amd"))
from qwen_tts.codec import CodecDecoder  # noqa: E402
from qwen_tts.weights import codec_specs, read_json, resolve_path, synthetic  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
T = int(sys.argv[2]) if len(sys.argv) > 2 else 256
dev = torch.device("cuda:0")
d = resolve_path("synthetic:1.7b-customvoice")
ccfg = read_json(os.path.join(d, "speech_tokenizer", "config.json"))
dec = CodecDecoder(ccfg, synthetic(codec_specs(ccfg), dev), dtype="bf16", device=dev)
codes = torch.randint(1, 2048, (B, T, 16), device=dev)
for _ in range(2):
    dec.decode(codes)
torch.cuda.synchronize()
n = 5
t0 = time.perf_counter()
for _ in range(n):
    w = dec.decode(codes)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / n
print(f"codec decode B={B} T={T}: {dt * 1e3:.2f} ms  ({B * T * 1920 / 24000 / dt:.0f} audio-s/s)  "
      f"igemm={'off' if os.environ.get('QT_NO_IGEMM') == '1' else 'on'}", flush=True)
