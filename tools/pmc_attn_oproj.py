"""Eager launches of the code-predictor fused attention + o_proj (attn_oproj_k, 1.7B dims, B=8, 10 keys: the mean
step) for rocprofv3 --pmc passes: 4 sweeps over the 5 layers' distinct o_proj weights, as in a frame.
QT_PMC_KEYS overrides the cache position (keys = pos + 1)."""
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
B = int(os.environ.get("QT_PMC_B", "8"))
pos = int(os.environ.get("QT_PMC_KEYS", "10")) - 1
kc = [torch.randn(B, c.Hkv, 18, c.D, device=dev).to(torch.bfloat16) for _ in c.layers]
vc = [torch.randn(B, c.Hkv, 18, c.D, device=dev).to(torch.bfloat16) for _ in c.layers]
qkv = torch.randn(B, c.qkv_w, device=dev)
x = torch.randn(B, c.H, device=dev)
x16 = x.to(torch.bfloat16)
ws = torch.zeros(Kn.attn_oproj_ws_bytes(c.H, c.Hkv), dtype=torch.uint8, device=dev)
torch.cuda.synchronize()
for hs in (False, True):  # the (column group, row) form (attn_oproj_k), then the head-split form (attn_oproj_hs_k)
    for _ in range(4):
        for i, L in enumerate(c.layers):
            Kn.decode_attn_oproj(qkv, B, c.Hq, c.Hkv, c.D, L.q_norm, L.k_norm, c.eps, c.cos, c.sin, kc[i], vc[i], 18,
                                 L.o, x, const_pos=pos, x16=x16, ws=ws if hs else None)
torch.cuda.synchronize()
L0 = c.layers[0]
algo = (L0.o.w.numel() * 2 + B * c.Hkv * (pos + 1) * c.D * 2 * 2 + B * c.qkv_w * 4 + B * c.H * (4 + 4 + 2))
print("algorithmic bytes per launch", algo)
with open(os.path.join(REPO, "gpurun_out", "pmc_ao_meta.txt"), "w") as f:
    f.write(f"{_hip.BUILD_ID or ''} {algo} {B} {pos + 1}\n")
