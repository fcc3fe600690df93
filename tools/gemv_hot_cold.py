"""Decode GEMV (M = 8) at the talker / code-predictor shapes with weights cold (cycling through > 600 MB, every
launch streams HBM), Infinity-Cache resident (cycling through ~120 MB: more than the 32 MiB of L2, less than the
256 MiB Infinity Cache) and hot (one matrix re-read, L2-resident): how much of each launch is memory time."""
import os
import sys
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "qwen3-tts_amd"))
from qwen_tts import kernels as K, _hip  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from microbench import timed  # noqa: E402

dev = torch.device("cuda:0")


def main():
    K.gemm_workspace(dev)
    sk = int(os.environ.get("QT_HC_SPLITK", "0"))
    only_cold = os.environ.get("QT_HC_COLD_ONLY", "0") == "1"
    shapes = [("talker qkv", 4096, 2048, True, 0), ("talker o", 2048, 2048, False, 1),
              ("talker gate-up", 12288, 2048, True, 2), ("talker down", 2048, 6144, False, 1),
              ("cp qkv", 4096, 1024, True, 0), ("cp gate-up", 6144, 1024, True, 2), ("cp down", 1024, 3072, False, 1),
              ("cp lm_head", 2048, 1024, True, 0)]
    for name, N, Kk, rms, epi in shapes:
        nmat = max(2, int(600e6 // (N * Kk * 2)))
        Ws = [K.tile_linear(torch.randn(N, Kk, device=dev) * 0.02, torch.bfloat16) for _ in range(nmat)]
        A = torch.randn(8, Kk, device=dev).to(torch.bfloat16)  # production A: x16 shadow / att / SwiGLU out (bf16)
        out = torch.zeros(8, N, device=dev)
        ep = [_hip.EPI_STORE, _hip.EPI_ADD, _hip.EPI_SWIGLU][epi]
        o = out if ep != _hip.EPI_SWIGLU else torch.zeros(8, N // 2, device=dev, dtype=torch.bfloat16)
        it = {"i": 0}

        def cold():
            K.gemm(A, Ws[it["i"] % nmat], o, 8, Kk, N, rms=rms, eps=1e-6, epi=ep, splitk=sk)
            it["i"] += 1

        def hot():
            K.gemm(A, Ws[0], o, 8, Kk, N, rms=rms, eps=1e-6, epi=ep, splitk=sk)
        nm = max(2, int(120e6 // (N * Kk * 2)))  # > the 32 MiB of L2, < the 256 MiB Infinity Cache

        def mall():
            K.gemm(A, Ws[it["i"] % nm], o, 8, Kk, N, rms=rms, eps=1e-6, epi=ep, splitk=sk)
            it["i"] += 1
        mb = N * Kk * 2 / 1e6
        for lab, f in ((("cold", cold),) if only_cold else (("cold", cold), ("mall", mall), ("hot", hot))):
            us = timed(f, f"{name} {N}x{Kk} ({mb:.1f} MB) {lab}")
            print(f"{'':60s} -> {mb * 1e3 / us:8.1f} GB/s", flush=True)
        del Ws


if __name__ == "__main__":
    main()
