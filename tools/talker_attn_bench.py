"""Talker decode attention (qt_decode_attention: q/k norm + RoPE + KV append + GQA attention) at the 1.7B dims,
B = 8, over cache lengths seen in the bench (prompt ~210 + up to 256 frames), split-KV 1 / 2 / 4."""
import os
import sys
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "qwen3-tts_amd"))
from qwen_tts import kernels as K  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from microbench import timed  # noqa: E402

dev = torch.device("cuda:0")


def main():
    B, hq, hkv, D = 8, 16, 8, 128
    Ls = [int(x) for x in os.environ.get("ATTN_L", "138,210,267,340,466").split(",")]
    Lmax = max(Ls) + 8
    nl = 28  # distinct layer caches: every launch streams its keys from HBM / MALL as in a frame
    kc = [torch.randn(B, hkv, Lmax, D, device=dev).to(torch.bfloat16) for _ in range(nl)]
    vc = [torch.randn(B, hkv, Lmax, D, device=dev).to(torch.bfloat16) for _ in range(nl)]
    qkv = torch.randn(B, (hq + 2 * hkv) * D, device=dev)
    qn = torch.ones(D, device=dev)
    cos, sin = K.rope_tables(D, 1e6, Lmax + 8, dev)
    att = torch.zeros(B, hq * D, device=dev, dtype=torch.bfloat16)
    i32 = lambda t: torch.as_tensor(t, dtype=torch.int32, device=dev)  # noqa: E731
    rb, zero = i32(range(B)), i32([0] * B)
    for L in Ls:
        pos = i32([L - 1] * B)
        for ns in [int(x) for x in os.environ.get("ATTN_NS", "1,2,4").split(",")]:
            ws = torch.zeros(K.decode_attn_ws_bytes(B, hq, hkv, D, ns), dtype=torch.uint8, device=dev) if ns > 1 else None
            it = {"i": 0}

            def f():
                i = it["i"] % nl
                it["i"] += 1
                K.decode_attention(qkv, B, hq, hkv, D, qn, qn, 1e-6, cos, sin, pos, rb, pos, zero, kc[i], vc[i], Lmax,
                                   att, nsplit=ns, ws=ws)
            us = timed(f, f"talker decode attention L={L} nsplit={ns}")
            print(f"{'':60s} -> {B * hkv * L * D * 2 * 2 / us / 1e3:8.1f} GB/s (KV bytes)", flush=True)


if __name__ == "__main__":
    main()
