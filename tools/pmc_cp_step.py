"""Eager launches of the code-predictor step engine (cp_step_k, 1.7B dims, B=8) for rocprofv3 --pmc / --kernel-trace
passes: 4 sweeps over the 14 decode steps of a frame (cache positions 2..15, lm_head 1..14), one workspace.
Writes gpurun_out/pmc_cs_meta.txt = "<build id> <algorithmic bytes per launch (mean over the 14 steps)> <B>" for
tools/pmc_kernel_reduce.py."""
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
cc = cfg["talker_config"]["code_predictor_config"]
pre = "talker.code_predictor.model"
specs = [(n, s) for n, s in talker_specs(cfg) if n.startswith(pre + ".layers.") or n == pre + ".norm.weight"]
W = synthetic(specs, dev)
c = _Stack(W, pre, cc, torch.bfloat16, dev, 18)
del W
B, Lmax, V = int(os.environ.get("QT_PMC_B", "8")), 18, cc["vocab_size"]
g = torch.Generator(device="cpu").manual_seed(5)
lm = [Kn.tile_linear((torch.randn(V, c.H, generator=g) * 0.02).to(dev), torch.bfloat16) for _ in range(15)]
kc = [torch.randn(B, c.Hkv, Lmax, c.D, device=dev).to(torch.bfloat16) for _ in c.layers]
vc = [torch.randn(B, c.Hkv, Lmax, c.D, device=dev).to(torch.bfloat16) for _ in c.layers]
qkv = torch.randn(B, c.qkv_w, device=dev)
x = torch.randn(B, c.H, device=dev)
logits = torch.empty(B, V, device=dev)
ws = torch.zeros(Kn.cp_step_ws_bytes(), dtype=torch.uint8, device=dev)
steps = list(range(1, 15))
torch.cuda.synchronize()
for _ in range(4):
    for s in steps:
        Kn.cp_step(c.layers, lm[s], x, qkv, B, kc, vc, Lmax, s + 1, c.cos, c.sin, c.eps, logits, ws)
torch.cuda.synchronize()
assert int(ws[:4].view(torch.int32).item()) == 0, "hand-off flag set"
nb = lambda Wt: Wt.w.numel() * Wt.w.element_size()  # noqa: E731
# layer 0's q/k/v weights are never read by a decode step (its rows come in through qkv0)
wb = sum(nb(L.o) + nb(L.gu) + nb(L.down) + (nb(L.qkv) if i > 0 else 0) for i, L in enumerate(c.layers))
kv = sum(len(c.layers) * B * c.Hkv * c.D * 2 * (2 * (s + 1) + 2) for s in steps) / len(steps)
algo = int(wb + lm[1].w.numel() * 2 + kv + B * (c.H + c.qkv_w + V) * 4)
print("algorithmic bytes per launch", algo)
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
with open(os.path.join(REPO, "gpurun_out", "pmc_cs_meta.txt"), "w") as f:
    f.write(f"{_hip.BUILD_ID or ''} {algo} {B}\n")
