"""Debug / A-B harness for qt_cp_step (the code-predictor step engine): engine vs the launch chain for 1..5 layers,
repeated launches on one workspace and on fresh workspaces, launch counter and error flag after each launch.
    python tools/ce_debug.py"""
import os
import sys

import torch

DBG = 6 * 5 * 16 * 4096 * 4  # cp_engine.hip DBG_BYTES: [layer][kind][token row][4096] fp32 stage records

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "qwen3-tts_amd"), os.path.join(REPO, "tests")]
from test_gpu_cp_engine import _chain, _cp_stack, _inputs, _rel  # noqa: E402
from qwen_tts import kernels as Kn  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    st, lm, g = _cp_stack(dev)
    all_layers = list(st.layers)
    Lmax = 18
    for nl in (1, 2, 5):
        st.layers = all_layers[:nl]
        st.n_layers = nl
        for R, pos in ((8, 2), (8, 9)):
            x, x16, qkv0, kc, vc = _inputs(st, R, Lmax, g, dev)
            ref = _chain(st, lm, x.clone(), x16.clone(), qkv0, [k.clone() for k in kc], [v.clone() for v in vc], R,
                         Lmax, pos, dev)
            ws = torch.zeros(Kn.cp_step_ws_bytes(), dtype=torch.uint8, device=dev)
            res = []
            for it in range(4):
                fresh = it == 3
                w = torch.zeros_like(ws) if fresh else ws
                logits = torch.full((R, lm.N), float("nan"), device=dev)
                Kn.cp_step(st.layers, lm, x, qkv0, R, [k.clone() for k in kc], [v.clone() for v in vc], Lmax, pos,
                           st.cos, st.sin, st.eps, logits, w)
                torch.cuda.synchronize()
                ep = int(w[4:8].view(torch.int32).item())
                err = int(w[:4].view(torch.int32).item())
                res.append(logits)
                print(f"nl={nl} R={R} pos={pos} launch {it}{' (fresh ws)' if fresh else ''}: rel vs chain "
                      f"{_rel(logits, ref):.3e} epoch {ep} err {err} finite {bool(torch.isfinite(logits).all())} "
                      f"same-as-first {bool(torch.equal(logits, res[0]))}", flush=True)
    st.layers = all_layers
    st.n_layers = len(all_layers)


if __name__ == "__main__" and not (os.environ.get("CE_LAYER0") or os.environ.get("CE_STAMPS") or os.environ.get("CE_TIME")
                               or os.environ.get("CE_PF_STAMPS")):
    main()


def layer0():
    """Layer-0 intermediates of the engine (workspace with the debug tail) vs the launch-chain kernels."""
    from qwen_tts import _hip
    dev = torch.device("cuda:0")
    st, lm, g = _cp_stack(dev)
    R, pos, Lmax = 8, 5, 18
    x, x16, qkv0, kc, vc = _inputs(st, R, Lmax, g, dev)
    L0 = st.layers[0]
    # chain intermediates
    att = torch.empty(R, st.Hq * st.D, dtype=torch.bfloat16, device=dev)
    i32 = lambda t: torch.as_tensor(t, dtype=torch.int32, device=dev)  # noqa: E731
    posv, rb, zero = i32([pos] * R), i32(range(R)), i32([0] * R)
    Kn.decode_attention(qkv0, R, st.Hq, st.Hkv, st.D, L0.q_norm, L0.k_norm, st.eps, st.cos, st.sin, posv, rb, posv, zero,
                        kc[0].clone(), vc[0].clone(), Lmax, att, const_pos=pos)
    xa = x.clone()
    xa16 = x16.clone()
    Kn.gemm(att, L0.o, xa, R, st.Hq * st.D, st.H, epi=_hip.EPI_ADD, out2=xa16)
    h = torch.empty(R, st.I, dtype=torch.bfloat16, device=dev)
    Kn.gemm(xa16, L0.gu, h, R, st.H, st.I, rms=True, eps=st.eps, epi=_hip.EPI_SWIGLU)
    xm = xa.clone()
    Kn.gemm(h, L0.down, xm, R, st.I, st.H, epi=_hip.EPI_ADD)
    n = Kn.cp_step_ws_bytes() + int(_hip.lib().qt_cp_step_dbg_bytes())
    for it in range(3):
        ws = torch.zeros(n, dtype=torch.uint8, device=dev)
        logits = torch.full((R, lm.N), float("nan"), device=dev)
        Kn.cp_step(st.layers[:1], lm, x, qkv0, R, [k.clone() for k in kc], [v.clone() for v in vc], Lmax, pos, st.cos,
                   st.sin, st.eps, logits, ws)
        torch.cuda.synchronize()
        d = ws[Kn.cp_step_ws_bytes():Kn.cp_step_ws_bytes() + DBG].view(torch.float32).view(6, 5, 16, 4096)[0]
        print(f"launch {it}: att rel {_rel(d[3, :R, :2048], att.float()):.3e}  x_attn rel {_rel(d[0, :R, :1024], xa):.3e}  "
              f"h rel {_rel(d[1, :R, :3072], h.float()):.3e}  x_mlp rel {_rel(d[2, :R, :1024], xm):.3e}", flush=True)
        for name, a, b in (("att", d[3, :R, :2048], att.float()), ("x_attn", d[0, :R, :1024], xa),
                           ("h", d[1, :R, :3072], h.float())):
            bad = ((a - b).abs() > 0.05 * b.abs().max()).nonzero()
            if bad.numel():
                print(f"   {name}: {bad.shape[0]} bad entries, first {bad[:8].tolist()}")


if __name__ == "__main__" and os.environ.get("CE_LAYER0"):
    layer0()


EVENTS = ["P1 wait", "x16(1) in", "qkv pub", "qkv in", "attn done", "part pub", "part in", "x16(0) pub", "x16(0) in",
          "h pub", "h in", "x16(1) pub"]


def stamps(R=8, reps=3):
    """Per-phase timestamps (s_memrealtime, 10 ns) of 14 consecutive engine launches (cache positions 2..15), as a
    frame issues them: per layer and event the median / max over blocks, microseconds from the launch's first block."""
    from qwen_tts import _hip
    import numpy as np
    dev = torch.device("cuda:0")
    st, lm, g = _cp_stack(dev)
    Lmax = 18
    x, x16, qkv0, kc, vc = _inputs(st, R, Lmax, g, dev)
    nws = Kn.cp_step_ws_bytes()
    n = nws + int(_hip.lib().qt_cp_step_dbg_bytes())
    ws = torch.zeros(n, dtype=torch.uint8, device=dev)
    logits = torch.empty(R, lm.N, device=dev)
    dbg_off = nws + DBG
    tot = []
    for rep in range(reps):
        for pos in range(2, 16):
            Kn.cp_step(st.layers, lm, x, qkv0, R, kc, vc, Lmax, pos, st.cos, st.sin, st.eps, logits, ws)
            torch.cuda.synchronize()
            t = ws[dbg_off:].view(torch.int64).view(256, 128).cpu().numpy().astype(np.float64) * 0.01  # us
            t0 = t[:, 0].min()
            tot.append(t[:, 1].max() - t0)
            if rep == reps - 1 and pos == 9:
                print(f"launch at pos {pos}: first block start -> last block end {t[:, 1].max() - t0:.2f} us; start "
                      f"spread {t[:, 0].max() - t0:.2f} us")
                for l in range(st.n_layers):
                    row = []
                    for k, name in enumerate(EVENTS):
                        v = t[:, 2 + 12 * l + k]
                        if l == 0 and k < 3:
                            continue
                        row.append(f"{name} {np.median(v) - t0:6.2f}/{v.max() - t0:6.2f}")
                    print(f"  layer {l}: " + " | ".join(row))
                subs = {0: "P1 mfma", 1: "P1 red_put", 2: "P1 barrier", 3: "qkv stores", 4: "qkv drained",
                        10: "P3 start", 11: "P3 dma waited", 12: "P3 mfma", 13: "P3 red_put", 14: "P3 barrier",
                        15: "P3 swiglu", 16: "P3 barrier2", 17: "h stores", 18: "h drained", 20: "P4 wait start",
                        21: "P4 staged", 22: "P4 barrier", 23: "P4 dma waited", 24: "P4 mfma+red", 25: "P4 barrier2"}
                print("  layer 2 sub-phases: " + " | ".join(
                    f"{n} {np.median(t[:, 64 + k]) - t0:6.2f}" for k, n in subs.items()))
    print(f"kernel time (first start -> last end) over {len(tot)} launches: median {np.median(tot):.2f} us, "
          f"min {np.min(tot):.2f}")


if __name__ == "__main__" and os.environ.get("CE_STAMPS"):
    stamps()


def timing(R=8, reps=50):
    """Device time per launch of 14 consecutive engine launches (cache positions 2..15) captured in one HIP graph,
    HIP events on the capture stream (no stamps: the product library)."""
    dev = torch.device("cuda:0")
    st, lm, g = _cp_stack(dev)
    Lmax = 18
    x, x16, qkv0, kc, vc = _inputs(st, R, Lmax, g, dev)
    ws = torch.zeros(Kn.cp_step_ws_bytes(), dtype=torch.uint8, device=dev)
    logits = torch.empty(R, lm.N, device=dev)

    def run():
        for pos in range(2, 16):
            Kn.cp_step(st.layers, lm, x, qkv0, R, kc, vc, Lmax, pos, st.cos, st.sin, st.eps, logits, ws)
    s = torch.cuda.Stream(device=dev)
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        run()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr, stream=s):
            run()
        gr.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(reps):
            gr.replay()
        e1.record(s)
    torch.cuda.synchronize()
    print(f"graph of 14 launches x {reps}: {e0.elapsed_time(e1) * 1e3 / (14 * reps):.2f} us per launch, "
          f"error flag {int(ws[:4].view(torch.int32).item())}")


if __name__ == "__main__" and os.environ.get("CE_TIME"):
    timing()


def pf_stamps(R=8, reps=3):
    """Per-phase timestamps of the 2-token prefill launch (qt_cp_prefill), as stamps() (layer 0 has its q/k/v phase)."""
    from qwen_tts import _hip
    import numpy as np
    dev = torch.device("cuda:0")
    st, lm, g = _cp_stack(dev)
    Lmax = 18
    x = torch.randn(2 * R, st.H, generator=g).to(dev)
    kc = [torch.zeros(R, st.Hkv, Lmax, st.D, device=dev, dtype=torch.bfloat16) for _ in st.layers]
    vc = [torch.zeros(R, st.Hkv, Lmax, st.D, device=dev, dtype=torch.bfloat16) for _ in st.layers]
    nws = Kn.cp_step_ws_bytes()
    ws = torch.zeros(nws + int(_hip.lib().qt_cp_step_dbg_bytes()), dtype=torch.uint8, device=dev)
    logits = torch.empty(R, lm.N, device=dev)
    dbg_off = nws + DBG
    tot = []
    for rep in range(reps * 5):
        Kn.cp_prefill(st.layers, lm, x, R, kc, vc, Lmax, st.cos, st.sin, st.eps, logits, ws)
        torch.cuda.synchronize()
        t = ws[dbg_off:].view(torch.int64).view(256, 128).cpu().numpy().astype(np.float64) * 0.01
        t0 = t[:, 0].min()
        tot.append(t[:, 1].max() - t0)
    print(f"prefill launch: first block start -> last block end {t[:, 1].max() - t0:.2f} us; start spread "
          f"{t[:, 0].max() - t0:.2f} us")
    for l in range(st.n_layers):
        print(f"  layer {l}: " + " | ".join(f"{n} {np.median(t[:, 2 + 12 * l + k]) - t0:6.2f}/"
                                            f"{t[:, 2 + 12 * l + k].max() - t0:6.2f}" for k, n in enumerate(EVENTS)))
    print(f"kernel time over {len(tot)} launches: median {np.median(tot):.2f} us, min {np.min(tot):.2f}")


if __name__ == "__main__" and os.environ.get("CE_PF_STAMPS"):
    pf_stamps()
