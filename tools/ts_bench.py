"""Talker decode step: qt_talker_step (one launch for all layers) vs the per-layer launches (attention + qt_talker_tail,
and attention + 4 GEMVs), 1.7B talker dims, 28 layers of seeded random weights, B rows at ~L keys; HIP graphs
replayed between HIP events.  With the probe library and TS_STAMPS=1: per-layer phase stamps of one launch.
    python tools/ts_bench.py [B] [keys]"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "qwen3-tts_amd"), os.path.join(REPO, "tests")]
from qwen_tts import _hip, kernels as Kn  # noqa: E402
from qwen_tts.talker import _scratch  # noqa: E402
from test_gpu_talker_step import _caches, _stack  # noqa: E402
from tt_bench import graph_us  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    keys = int(sys.argv[2]) if len(sys.argv) > 2 else 267
    st = _stack(dev, 28)
    Lmax = keys + 8
    i32 = lambda v: torch.full((B,), v, dtype=torch.int32, device=dev)  # noqa: E731
    meta = {"rope_pos": i32(keys - 1), "kv_pos": i32(keys - 1), "row_start": i32(0),
            "row_batch": torch.arange(B, dtype=torch.int32, device=dev), "nsplit": 1}
    kc, vc = _caches(st, B, Lmax, dev, 3)
    x = torch.randn(B, st.H, device=dev)
    x16 = x.to(torch.bfloat16)
    sc = _scratch(B, st, dev)
    sc_t = dict(_scratch(B, st, dev), tt_ws=torch.zeros(Kn.talker_tail_ws_bytes(), dtype=torch.uint8, device=dev))
    ws = torch.zeros(Kn.talker_step_ws_bytes() + int(_hip.lib().qt_talker_step_stamp_bytes()), dtype=torch.uint8,
                     device=dev)
    tab = Kn.talker_step_table(st.layers, kc, vc, dev)

    def chain():
        st.forward(x, B, meta, (kc, vc), sc, Lmax, Lmax, decode=True, x16=x16)

    def tail():
        st.forward(x, B, meta, (kc, vc), sc_t, Lmax, Lmax, decode=True, x16=x16)

    def step():
        Kn.talker_step(tab, st.n_layers, B, x, Lmax, st.cos, st.sin, meta["rope_pos"], meta["kv_pos"],
                       meta["row_start"], meta["row_batch"], st.eps, ws)

    q = [torch.empty(B, st.qkv_w, device=dev) for _ in range(2)]

    def step_layers():
        Kn.gemm(x16, st.layers[0].qkv, q[0], B, st.H, st.qkv_w, rms=True, eps=st.eps)
        for li in range(st.n_layers):
            Kn.talker_step(tab, 1, B, x, Lmax, st.cos, st.sin, meta["rope_pos"], meta["kv_pos"], meta["row_start"],
                           meta["row_batch"], st.eps, ws, first_layer=li, total_layers=st.n_layers,
                           qkv_in=q[li % 2], qkv_out=q[(li + 1) % 2] if li + 1 < st.n_layers else None)

    att = [torch.empty(B, st.Hq * st.D, dtype=torch.bfloat16, device=dev) for _ in range(2)]

    def step_att():
        Kn.gemm(x16, st.layers[0].qkv, q[0], B, st.H, st.qkv_w, rms=True, eps=st.eps)
        L0 = st.layers[0]
        Kn.decode_attention(q[0], B, st.Hq, st.Hkv, st.D, L0.q_norm, L0.k_norm, st.eps, st.cos, st.sin, meta["rope_pos"],
                            meta["row_batch"], meta["kv_pos"], meta["row_start"], kc[0], vc[0], Lmax, att[0])
        for li in range(st.n_layers):
            Kn.talker_step(tab, 1, B, x, Lmax, st.cos, st.sin, meta["rope_pos"], meta["kv_pos"], meta["row_start"],
                           meta["row_batch"], st.eps, ws, first_layer=li, total_layers=st.n_layers,
                           att_in=att[li % 2], att_out=att[(li + 1) % 2] if li + 1 < st.n_layers else None)

    cases = (("chain: attention + 4 GEMVs per layer", chain), ("attention + qt_talker_tail per layer", tail),
             ("qt_talker_step per layer: o_proj .. next attention", step_att),
             ("qt_talker_step (one launch)", step), ("qt_talker_step per layer (q/k/v GEMV + 28 launches)",
                                                    step_layers)) * 2
    if os.environ.get("TS_ONLY"):
        cases = (("qt_talker_step per layer: o_proj .. next attention", step_att),) * 2
    for name, fn in cases:
        us = graph_us(fn, 5, dev)
        print(f"B={B} keys={keys} {name}: {us:.1f} us per step = {us / 28:.2f} us per layer", flush=True)
    print("error flag", int(ws[:4].view(torch.int32).item()))
    if os.environ.get("TS_STAMPS") and _hip.PROBE:
        import numpy as np
        step()
        torch.cuda.synchronize()
        t = ws[Kn.talker_step_ws_bytes():].view(torch.int64).view(256, 32, 16).cpu().numpy().astype(np.float64) * 0.01
        t0 = t[:, 0, 0].min()
        names = ["layer", "q staged", "q pub", "att pub", "att staged", "o pub", "x1 staged", "h pub", "h staged",
                 "down pub"]
        for l in (0, 1, 2, 13, 27):
            print(f"  layer {l:2d}: " + " | ".join(f"{n} {np.median(t[:, l, k]) - t0:7.2f}/{t[:, l, k].max() - t0:7.2f}"
                                                  for k, n in enumerate(names)))


if __name__ == "__main__":
    main()
