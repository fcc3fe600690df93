"""A/B of decode-GEMV variants on the production shapes (M = 8, bf16 weights, cold: > 256 MiB of distinct matrices
cycled so every launch streams HBM).  Variants are chosen by the QT_GEMV_* env switches read once by the library,
so run one process per setting:

    QT_GEMV_U=8 python tools/gemv_ab.py      (measured variants: profiles/r01_gemv_variants_ab.jsonl)
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "qwen3-tts_amd"))
from qwen_tts import kernels as K, _hip  # noqa: E402

dev = torch.device("cuda:0")
N_LAUNCH = 200


def timed(fn):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(N_LAUNCH):
                fn()
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (10 * N_LAUNCH)


def main():
    K.gemm_workspace(dev)
    # (name, N, K, kind): kinds as the talker / code predictor issue them in bf16 mode
    shapes = [("talker_gate_up", 12288, 2048, "swiglu"), ("talker_qkv", 4096, 2048, "rms"),
              ("talker_o", 2048, 2048, "add_bf16a"), ("talker_down", 2048, 6144, "add_bf16a"),
              ("cp_gate_up", 6144, 1024, "swiglu"), ("cp_qkv", 4096, 1024, "rms"), ("cp_o", 1024, 2048, "add_bf16a"),
              ("cp_down", 1024, 3072, "add_bf16a"), ("codec_head", 3072, 2048, "rms")]
    res = {"env": {k: v for k, v in os.environ.items() if k.startswith("QT_")}}
    for name, Nn, Kk, kind in shapes:
        nmat = max(2, int(600e6 // (Nn * Kk * 2)))
        if kind == "swiglu":
            Ws = [K.tile_swiglu(torch.randn(Nn // 2, Kk, device=dev) * 0.02, torch.randn(Nn // 2, Kk, device=dev) * 0.02,
                                torch.bfloat16) for _ in range(nmat)]
        else:
            Ws = [K.tile_linear(torch.randn(Nn, Kk, device=dev) * 0.02, torch.bfloat16) for _ in range(nmat)]
        A32 = torch.randn(8, Kk, device=dev)
        A16 = A32.to(torch.bfloat16)
        it = {"i": 0}
        if kind == "swiglu":
            out = torch.zeros(8, Nn // 2, dtype=torch.bfloat16, device=dev)

            def f():
                K.gemm(A32, Ws[it["i"] % nmat], out, 8, Kk, Nn // 2, rms=True, eps=1e-6, epi=_hip.EPI_SWIGLU)
                it["i"] += 1
            abytes = 8 * Kk * 4 + 8 * (Nn // 2) * 2
        elif kind == "rms":
            out = torch.zeros(8, Nn, device=dev)

            def f():
                K.gemm(A32, Ws[it["i"] % nmat], out, 8, Kk, Nn, rms=True, eps=1e-6)
                it["i"] += 1
            abytes = 8 * Kk * 4 + 8 * Nn * 4
        else:
            out = torch.zeros(8, Nn, device=dev)

            def f():
                K.gemm(A16, Ws[it["i"] % nmat], out, 8, Kk, Nn, epi=_hip.EPI_ADD)
                it["i"] += 1
            abytes = 8 * Kk * 2 + 2 * 8 * Nn * 4
        us = timed(f)
        res[name] = dict(us=round(us, 3), gbs=round((Nn * Kk * 2 + abytes) / us / 1e3, 1))
        del Ws
        torch.cuda.empty_cache()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
