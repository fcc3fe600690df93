"""Talker prefill linears at streaming-text prompt sizes (M = 8 x ~10 rows), 1.7B dims: per-launch time of each
shape on the path qt_gemm picks (QT_IGEMM_MIN_M moves the implicit-GEMM threshold, QT_GEMV_MAX_M the row-grouped
decode GEMV's, for A/B)."""
import os
import sys
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "qwen3-tts_amd"))
from qwen_tts import kernels as K, _hip  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from microbench import timed  # noqa: E402

dev = torch.device("cuda:0")
K.gemm_workspace(dev)  # the engine passes one (split-K of the decode GEMV and of gemm_pf2_k)


def main():
    # the RMS GEMMs read the bf16 residual shadow when the prefill runs on gemm_pf_k (QT_PF != 0), else fp32 x
    xdt = torch.float32 if os.environ.get("QT_PF", "1") == "0" else torch.bfloat16
    shapes = [("qkv", 4096, 2048, True, 0, xdt), ("o", 2048, 2048, False, 1, torch.bfloat16),
              ("gate-up", 12288, 2048, True, 2, xdt), ("down", 2048, 6144, False, 1, torch.bfloat16)]
    if os.environ.get("QT_PB_DIMS") == "0.6b":  # 0.6B talker / 1.7B code predictor (hidden 1024)
        shapes = [("qkv", 4096, 1024, True, 0, xdt), ("o", 1024, 2048, False, 1, torch.bfloat16),
                  ("gate-up", 6144, 1024, True, 2, xdt), ("down", 1024, 3072, False, 1, torch.bfloat16)]
    for M in [int(m) for m in os.environ.get("QT_PB_M", "24,48,80,112,160,256").split(",")]:
        for name, N, Kk, rms, epi, adt in shapes:
            nmat = max(2, int(600e6 // (N * Kk * 2)))
            Ws = [K.tile_linear(torch.randn(N, Kk, device=dev) * 0.02, torch.bfloat16) for _ in range(nmat)]
            A = torch.randn(M, Kk, device=dev).to(adt)
            ep = [_hip.EPI_STORE, _hip.EPI_ADD, _hip.EPI_SWIGLU][epi]
            o = torch.zeros(M, N, device=dev) if ep != _hip.EPI_SWIGLU else torch.zeros(M, N // 2, device=dev,
                                                                                          dtype=torch.bfloat16)
            it = {"i": 0}

            def f():
                K.gemm(A, Ws[it["i"] % nmat], o, M, Kk, o.shape[1], rms=rms, eps=1e-6, epi=ep)
                it["i"] += 1
            timed(f, f"prefill {name} M={M} {N}x{Kk}")
            del Ws


if __name__ == "__main__":
    main()
