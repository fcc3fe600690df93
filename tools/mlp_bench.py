"""Fused decode MLP (qt_mlp_decode) vs the two-GEMV path, cold weights, graphs of launches (same run)."""
import os
import sys
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "qwen3-tts_amd"))
from qwen_tts import kernels as K, _hip  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from microbench import timed  # noqa: E402

dev = torch.device("cuda:0")
K.gemm_workspace(dev)
for (M, H, I) in [(8, 1024, 3072), (8, 2048, 6144)]:
    nmat = max(2, int(600e6 // (3 * H * I * 2)))
    mats = [(K.tile_swiglu(torch.randn(I, H, device=dev) * 0.03, torch.randn(I, H, device=dev) * 0.03, torch.bfloat16),
             K.tile_linear(torch.randn(H, I, device=dev) * 0.03, torch.bfloat16)) for _ in range(nmat)]
    x = torch.randn(M, H, device=dev)
    h = torch.empty(M, I, dtype=torch.bfloat16, device=dev)
    ws = torch.zeros(K.mlp_ws_bytes(M, H, I), dtype=torch.uint8, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    it = {"i": 0}

    def two():
        gu, dn = mats[it["i"] % nmat]
        K.gemm(x, gu, h, M, H, I, rms=True, eps=1e-6, epi=_hip.EPI_SWIGLU)
        K.gemm(h, dn, x, M, I, H, epi=_hip.EPI_ADD)
        it["i"] += 1

    def fused():
        gu, dn = mats[it["i"] % nmat]
        K.mlp_decode(x, M, H, I, gu, dn, 1e-6, ws, err)
        it["i"] += 1
    timed(two, f"MLP two GEMVs M={M} H={H} I={I} (per pair = 2 launches)")
    timed(fused, f"MLP fused    M={M} H={H} I={I}")
    del mats
