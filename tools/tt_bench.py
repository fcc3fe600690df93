"""Talker decode-layer tail: qt_talker_tail (one persistent launch per layer) vs the launch chain it replaces (o_proj,
gate/up, down, next q/k/v GEMVs), 1.7B talker shapes, 28 layers of distinct random weights (every launch streams its
weights from HBM, as in a frame), B rows; HIP graphs replayed between HIP events.  With the probe library and
TT_STAMPS=1: per-phase timestamps of one launch (median / max over blocks).
    python tools/tt_bench.py [B] [H]   (H 2048: the 1.7B talker, I 6144; H 1024: the 0.6B talker, I 3072)"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "qwen3-tts_amd"), os.path.join(REPO, "tests")]
from qwen_tts import _hip, kernels as Kn  # noqa: E402
from test_gpu_talker_tail import _L, HQ, D, QKV  # noqa: E402


def graph_us(run, reps, dev):
    s = torch.cuda.Stream(device=dev)
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        run()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            run()
        g.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(reps):
            g.replay()
        e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    dev = torch.device("cuda:0")
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    H = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
    I = 3 * H
    nl = 28
    g = torch.Generator().manual_seed(1)
    layers = [_L(g, dev, H, I) for _ in range(nl + 1)]
    att = torch.randn(B, HQ * D, device=dev).to(torch.bfloat16)
    x = torch.randn(B, H, device=dev)
    x16 = x.to(torch.bfloat16)
    h = torch.empty(B, I, dtype=torch.bfloat16, device=dev)
    qkv = torch.empty(B, QKV, device=dev)
    ws = torch.zeros(Kn.talker_tail_ws_bytes() + int(_hip.lib().qt_talker_tail_stamp_bytes()), dtype=torch.uint8,
                     device=dev)
    eps = 1e-6

    def chain():
        for i in range(nl):
            L, Ln = layers[i], layers[i + 1]
            Kn.gemm(att, L.o, x, B, HQ * D, H, epi=_hip.EPI_ADD, out2=x16)
            Kn.gemm(x16, L.gu, h, B, H, I, rms=True, eps=eps, epi=_hip.EPI_SWIGLU)
            Kn.gemm(h, L.down, x, B, I, H, epi=_hip.EPI_ADD, out2=x16)
            Kn.gemm(x16, Ln.qkv, qkv, B, H, QKV, rms=True, eps=eps)

    def tail():
        for i in range(nl):
            Kn.talker_tail(att, x, B, layers[i], layers[i + 1], qkv, eps, ws)

    wb = sum(t.w.numel() * 2 for t in (layers[0].o, layers[0].gu, layers[0].down, layers[0].qkv))
    for name, fn in (("chain (4 GEMV launches)", chain), ("qt_talker_tail", tail), ("chain (4 GEMV launches)", chain),
                     ("qt_talker_tail", tail)):
        us = graph_us(fn, 5, dev) / nl
        print(f"H={H} B={B} {name}: {us:.2f} us per layer = {wb / (us * 1e-6) / 1e12:.2f} TB/s of weights", flush=True)
    print("error flag", int(ws[:4].view(torch.int32).item()))
    if os.environ.get("TT_STAMPS") and _hip.PROBE:
        import numpy as np
        Kn.talker_tail(att, x, B, layers[3], layers[4], qkv, eps, ws)
        torch.cuda.synchronize()
        t = ws[Kn.talker_tail_ws_bytes():].view(torch.int64)[:H // 8 * 32].view(H // 8, 32).cpu().numpy()
        t = t.astype(np.float64) * 0.01
        t0 = t[:, 0].min()
        names = ["start", "staged", "o done", "x1 in", "x16 staged", "h pub", "h in", "h staged", "down done",
                 "qkv staged", "end"]
        print("  " + " | ".join(f"{n} {np.median(t[:, k]) - t0:6.2f}/{t[:, k].max() - t0:6.2f}" for k, n in enumerate(names)))


if __name__ == "__main__":
    main()
