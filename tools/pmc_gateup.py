"""Eager launches of the roofline kernel (talker MLP gate-up decode GEMV, 1.7B dims, M=8) for rocprofv3 --pmc
passes: 3 sweeps over the 28 layers (distinct weights -> every launch streams HBM)."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "qwen3-tts_amd"))
from qwen_tts import _hip, kernels as Kn  # noqa: E402
from qwen_tts.talker import _Stack  # noqa: E402
from qwen_tts.weights import read_json, resolve_path, synthetic, talker_specs  # noqa: E402

dev = torch.device("cuda:0")
cfg = read_json(os.path.join(resolve_path("synthetic:1.7b-customvoice"), "config.json"))
tc = cfg["talker_config"]
specs = [(n, s) for n, s in talker_specs(cfg) if n.startswith("talker.model.layers.") or n == "talker.model.norm.weight"]
W = synthetic(specs, dev)
t = _Stack(W, "talker.model", tc, torch.bfloat16, dev, 64)
del W
B = 8
x = torch.randn(B, t.H, device=dev).to(torch.bfloat16)  # the bf16 residual shadow, as in the frame graph
h = torch.empty(B, t.I, dtype=torch.bfloat16, device=dev)
torch.cuda.synchronize()
for _ in range(3):
    for L in t.layers:
        Kn.gemm(x, L.gu, h, B, t.H, t.I, rms=True, eps=t.eps, epi=_hip.EPI_SWIGLU)
torch.cuda.synchronize()
print("weight bytes per launch", t.layers[0].gu.w.numel() * 2)
with open(os.path.join(REPO, "gpurun_out", "pmc_build_id.txt"), "w") as f:
    f.write(_hip.BUILD_ID or "")
