"""Eager launches of the talker decode-layer tail engine (talker_tail_k, 1.7B talker dims, B=8): 2 sweeps over 28
layers of distinct random weights, for rocprofv3 --pmc passes.  Writes gpurun_out/pmc_tt_meta.txt = "<build id>
<algorithmic bytes per launch> <B>" for tools/pmc_kernel_reduce.py."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "qwen3-tts_amd"), os.path.join(REPO, "tests")]
from qwen_tts import _hip, kernels as Kn  # noqa: E402
from test_gpu_talker_tail import _L, H, HQ, D, QKV  # noqa: E402

dev = torch.device("cuda:0")
B, nl = 8, 28
g = torch.Generator().manual_seed(1)
layers = [_L(g, dev) for _ in range(nl + 1)]
att = torch.randn(B, HQ * D, device=dev).to(torch.bfloat16)
x = torch.randn(B, H, device=dev)
qkv = torch.empty(B, QKV, device=dev)
ws = torch.zeros(Kn.talker_tail_ws_bytes(), dtype=torch.uint8, device=dev)
torch.cuda.synchronize()
for _ in range(2):
    for i in range(nl):
        Kn.talker_tail(att, x, B, layers[i], layers[i + 1], qkv, 1e-6, ws)
torch.cuda.synchronize()
assert int(ws[:4].view(torch.int32).item()) == 0, "hand-off flag set"
L0 = layers[0]
algo = int(sum(t.w.numel() * 2 for t in (L0.o, L0.gu, L0.down, L0.qkv)) + B * HQ * D * 2 + B * H * 8 + B * QKV * 4)
print("algorithmic bytes per launch", algo)
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
with open(os.path.join(REPO, "gpurun_out", "pmc_tt_meta.txt"), "w") as f:
    f.write(f"{_hip.BUILD_ID or ''} {algo} {B}\n")
