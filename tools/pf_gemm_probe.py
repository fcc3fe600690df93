"""Prefill GEMM probe: the 1.7B talker layer's four prefill linears at M rows on qt_gemm's own path (gemm_pf_k) next to
torch.matmul (hipBLASLt, plain bf16 GEMM, no fused prologue / epilogue) on the same shapes -- what a library GEMM
reaches here is the practical target.  Weights distinct per launch (28 layers' worth), HIP events around graph
replays.

    python tools/pf_gemm_probe.py [M ...]        (QT_PROBE_SHAPES=gate-up,down limits the shapes)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "qwen3-tts_amd"))
from qwen_tts import _hip, kernels as K  # noqa: E402

dev = torch.device("cuda:0")
SHAPES = [("qkv", 4096, 2048, True, _hip.EPI_STORE), ("o", 2048, 2048, False, _hip.EPI_ADD),
          ("gate-up", 12288, 2048, True, _hip.EPI_SWIGLU), ("down", 2048, 6144, False, _hip.EPI_ADD)]


def graph_us(fn, reps=5):
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        fn()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=st):
            fn()
        g.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            g.replay()
        e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    Ms = [int(x) for x in sys.argv[1:]] or [680, 1600]
    nl = 8
    for M in Ms:
        tot_ours = tot_lib = 0.0
        flops_tot = 0.0
        only = [x for x in os.environ.get("QT_PROBE_SHAPES", "").split(",") if x]
        for name, N, Kk, rms, epi in SHAPES:
            if only and name not in only:
                continue
            Wf = [torch.randn(N, Kk, device=dev) * 0.02 for _ in range(nl)]
            Wt = [K.tile_linear(w, torch.bfloat16) for w in Wf]
            Wb = [w.to(torch.bfloat16).t().contiguous() for w in Wf]  # [K][N] for A @ W
            del Wf
            pad = int(os.environ.get("QT_PROBE_LDA_PAD", "0"))  # A row stride K + pad elements
            A = torch.randn(M, Kk + pad, device=dev).to(torch.bfloat16)[:, :Kk]
            o = (torch.zeros(M, N // 2, device=dev, dtype=torch.bfloat16) if epi == _hip.EPI_SWIGLU else
                 torch.zeros(M, N, device=dev))
            o16 = torch.empty(M, N, device=dev, dtype=torch.bfloat16)

            def ours():
                for w in Wt:
                    K.gemm(A, w, o, M, Kk + pad, o.shape[1], rms=rms, eps=1e-6, epi=epi)

            def lib():
                for w in Wb:
                    torch.matmul(A, w, out=o16)
            t_o = graph_us(ours) / nl
            t_l = graph_us(lib) / nl
            fl = 2.0 * M * N * Kk
            flops_tot += fl
            tot_ours += t_o
            tot_lib += t_l
            print(f"M={M:5d} {name:8s} N={N:5d} K={Kk:5d}: qt_gemm {t_o:7.1f} us ({fl / t_o / 1e6:6.1f} TF/s)   "
                  f"torch.matmul {t_l:7.1f} us ({fl / t_l / 1e6:6.1f} TF/s)", flush=True)
            del Wt, Wb
        print(f"M={M:5d} layer: qt_gemm {tot_ours:7.1f} us ({flops_tot / tot_ours / 1e6:6.1f} TF/s)   "
              f"torch.matmul {tot_lib:7.1f} us ({flops_tot / tot_lib / 1e6:6.1f} TF/s)", flush=True)


if __name__ == "__main__":
    main()
