"""How far the chunked streaming decode (left context ctx frames + 1 lookahead frame) is from the one-shot
decode, on the 1.7B codec dims with seeded synthetic weights and random codes (fp32 and bf16)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "qwen3-tts_amd"))
from qwen_tts.codec import CodecDecoder  # noqa: E402
from qwen_tts.weights import codec_specs, read_json, resolve_path, synthetic  # noqa: E402

dev = torch.device("cuda:0")
ccfg = read_json(os.path.join(resolve_path("synthetic:1.7b-customvoice"), "speech_tokenizer", "config.json"))
W = synthetic(codec_specs(ccfg), dev)
T = 160
g = torch.Generator().manual_seed(0)
codes = torch.randint(1, 2048, (2, T, 16), generator=g).to(dev)
for dt in ("fp32", "bf16"):
    dec = CodecDecoder(ccfg, W, dtype=dt, device=dev)
    up = dec.total_upsample
    ref = dec.forward(codes)  # [2, 1920T - 555]
    for ctx in (25, 72, 150):
        pieces, s, first, step = [], 0, 12, 48
        e = first
        while s < T:
            last = e >= T
            e = min(e, T)
            c = min(ctx, s)
            w = dec.forward(codes[:, s - c:(T if last else e + 1)])
            n = up * (e - s) - (555 if last else 0)
            pieces.append(w[:, c * up:c * up + n])
            s, e = e, e + step
        got = torch.cat(pieces, 1)
        d = (got - ref).abs()
        rel = (got - ref).norm() / ref.norm()
        print(f"{dt} ctx={ctx:3d}: len {got.shape[1]} vs {ref.shape[1]}  max|diff| {d.max().item():.3e}  "
              f"rel-L2 {rel.item():.3e}  (ref rms {ref.pow(2).mean().sqrt().item():.3e})", flush=True)
