"""gemm_sk2_k numerics (run with QT_SK2=1): qt_gemm at 49..128 rows of the 1.7B talker prefill shapes (q/k/v with RMS,
o_proj with residual + bf16 shadow, gate-up SwiGLU) against a torch fp32 reference of the same bf16 operands, and
bitwise reproducibility over repeated calls / per-row independence of M."""
import os
import sys
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "qwen3-tts_amd"))
from qwen_tts import kernels as K, _hip  # noqa: E402

dev = torch.device("cuda:0")
K.gemm_workspace(dev)
g = torch.Generator().manual_seed(3)
worst = 0.0
for (name, N, Kk, rms, epi) in [("qkv", 4096, 2048, True, 0), ("o", 2048, 2048, False, 1), ("o4k", 2048, 4096, False, 1)]:
    Wf = (torch.randn(N, Kk, generator=g) * 0.02).to(dev)
    W = K.tile_linear(Wf, torch.bfloat16)
    Wb = Wf.to(torch.bfloat16).float()
    outs = {}
    for M in (49, 64, 96, 128, 96):
        A = torch.randn(128, Kk, generator=torch.Generator().manual_seed(7)).to(dev).to(torch.bfloat16)[:M]
        ref = A.float() @ Wb.t()
        if rms:
            ref = ref * torch.rsqrt(A.float().pow(2).mean(1, keepdim=True) + 1e-6)
        if epi == 0:
            o = torch.zeros(M, N, device=dev)
            K.gemm(A, W, o, M, Kk, N, rms=rms, eps=1e-6)
        else:
            x0 = torch.randn(128, N, generator=torch.Generator().manual_seed(9)).to(dev)[:M]
            o = x0.clone()
            o16 = torch.zeros(M, N, device=dev, dtype=torch.bfloat16)
            K.gemm(A, W, o, M, Kk, N, epi=_hip.EPI_ADD, out2=o16)
            assert torch.equal(o16, o.to(torch.bfloat16)), name
            ref = ref + x0
        err = (o - ref).abs().max().item() / max(ref.abs().max().item(), 1e-6)
        worst = max(worst, err)
        if M in outs:
            assert torch.equal(outs[M], o), f"{name} M={M}: not reproducible"
        outs[M] = o
        print(f"{name} M={M}: max rel err {err:.2e}", flush=True)
    assert torch.equal(outs[49], outs[128][:49]) and torch.equal(outs[96], outs[128][:96]), f"{name}: rows depend on M"
print("worst", worst)
assert worst < 1e-2
print("sk2 check ok")
