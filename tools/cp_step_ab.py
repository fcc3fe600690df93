"""A/B timing of the code-predictor step engine (qt_cp_step, 1.7B dims, B=8): the 14 decode steps of a frame (cache
positions 2..15) captured in one HIP graph, replayed between HIP events; prints us per launch (median of 5 x 20
replays).  Run once per library (QWEN3TTS_AMD_LIB=... QT_ALLOW_STALE_LIB=1 for an older build)."""
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
B, Lmax, V = int(os.environ.get("QT_AB_B", "8")), 18, cc["vocab_size"]
g = torch.Generator(device="cpu").manual_seed(5)
lm = [Kn.tile_linear((torch.randn(V, c.H, generator=g) * 0.02).to(dev), torch.bfloat16) for _ in range(15)]
kc = [torch.randn(B, c.Hkv, Lmax, c.D, device=dev).to(torch.bfloat16) for _ in c.layers]
vc = [torch.randn(B, c.Hkv, Lmax, c.D, device=dev).to(torch.bfloat16) for _ in c.layers]
qkv = torch.randn(B, c.qkv_w, device=dev)
x = torch.randn(B, c.H, device=dev)
logits = torch.empty(B, V, device=dev)
ws = torch.zeros(Kn.cp_step_ws_bytes(), dtype=torch.uint8, device=dev)
steps = list(range(1, 15))
st = torch.cuda.Stream()
st.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(st):
    def run():
        for s in steps:
            Kn.cp_step(c.layers, lm[s], x, qkv, B, kc, vc, Lmax, s + 1, c.cos, c.sin, c.eps, logits, ws)
    run()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr, stream=st):
        run()
    res = []
    for _ in range(6):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(20):
            gr.replay()
        e1.record(st)
        e1.synchronize()
        res.append(e0.elapsed_time(e1) * 1e3 / (20 * len(steps)))
torch.cuda.synchronize()
assert int(ws[:4].view(torch.int32).item()) == 0
res = sorted(res[1:])
print(f"{os.path.basename(_hip.LIB_PATH)} {_hip.BUILD_ID}: cp_step {res[len(res) // 2]:.2f} us per launch "
      f"(min {res[0]:.2f}, B={B})", flush=True)
