"""Per-launch cost of small decode kernels: graphs of N identical launches timed with HIP events."""
import os
import sys
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "qwen3-tts_amd"))
from qwen_tts import kernels as K, _hip  # noqa: E402

dev = torch.device("cuda:0")
N = 200


def timed(fn, label):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(N):
                fn()
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / (10 * N)
    print(f"{label:60s} {us:8.2f} us/launch", flush=True)
    return us


def main():
    ctr = torch.zeros(4, dtype=torch.int32, device=dev)
    timed(lambda: K.advance(ctr, 2), "advance (1 block, trivial)")
    K.gemm_workspace(dev)
    # cold weights: cycle through enough distinct matrices (> 256 MiB Infinity Cache) that every launch streams HBM;
    # split-K off (1) vs auto (0) vs forced factors, same box / same run (QT_GEMV_WPB env caps waves per block)
    shapes = [(1024, 1024), (2048, 1024), (1024, 2048), (4096, 1024), (6144, 1024), (1024, 3072), (2048, 2048),
              (4096, 2048), (3072, 2048), (12288, 2048), (2048, 6144)]
    for (Nn, Kk) in shapes:
        nmat = max(2, int(600e6 // (Nn * Kk * 2)))
        Ws = [K.tile_linear(torch.randn(Nn, Kk, device=dev) * 0.02, torch.bfloat16) for _ in range(nmat)]
        A = torch.randn(8, Kk, device=dev)
        out = torch.zeros(8, Nn, device=dev)
        for sk in (1, 0, 2, 4):  # 1 no split, 0 auto, n split-K
            for rms in ((False, True) if sk in (1, 0) else (False,)):
                it = {"i": 0}

                def f():
                    K.gemm(A, Ws[it["i"] % nmat], out, 8, Kk, Nn, splitk=sk, rms=rms, eps=1e-6)
                    it["i"] += 1
                us = timed(f, f"COLD gemv M=8 N={Nn} K={Kk} splitk={sk}{' rms' if rms else ''}")
                if not rms:
                    print(f"{'':60s} -> {Nn * Kk * 2 / us / 1e3:8.1f} GB/s")
        del Ws
    # rms GEMVs reading the residual stream as fp32 vs bf16 (gate/up + SwiGLU epilogue, qkv)
    for (Nn, Kk, epi) in [(12288, 2048, _hip.EPI_SWIGLU), (4096, 2048, _hip.EPI_STORE), (6144, 1024, _hip.EPI_SWIGLU),
                          (4096, 1024, _hip.EPI_STORE)]:
        nmat = max(2, int(600e6 // (Nn * Kk * 2)))
        Ws = [K.tile_linear(torch.randn(Nn, Kk, device=dev) * 0.02, torch.bfloat16) for _ in range(nmat)]
        for adt in (torch.float32, torch.bfloat16):
            A = torch.randn(8, Kk, device=dev).to(adt)
            out = torch.zeros(8, Nn, device=dev, dtype=torch.bfloat16)
            it = {"i": 0}

            def f():
                K.gemm(A, Ws[it["i"] % nmat], out, 8, Kk, Nn, rms=True, eps=1e-6, epi=epi)
                it["i"] += 1
            timed(f, f"COLD gemv rms A={str(adt)[6:]} M=8 N={Nn} K={Kk}")
        del Ws
    # bf16 activations (attention / SwiGLU outputs feeding o-proj / down-proj in bf16 mode), residual add
    for (Nn, Kk) in [(1024, 3072), (1024, 2048), (2048, 6144), (2048, 2048)]:
        nmat = max(2, int(600e6 // (Nn * Kk * 2)))
        Ws = [K.tile_linear(torch.randn(Nn, Kk, device=dev) * 0.02, torch.bfloat16) for _ in range(nmat)]
        A = torch.randn(8, Kk, device=dev).bfloat16()
        out = torch.zeros(8, Nn, device=dev)
        for sk in (1, 2, 4, 8, 0):
            it = {"i": 0}

            def f():
                K.gemm(A, Ws[it["i"] % nmat], out, 8, Kk, Nn, splitk=sk, epi=_hip.EPI_ADD)
                it["i"] += 1
            timed(f, f"COLD gemv bf16-A add M=8 N={Nn} K={Kk} splitk={sk}")
        del Ws
    lg = torch.randn(8, 3072, device=dev)
    tok = torch.zeros(8, dtype=torch.int32, device=dev)
    step = torch.zeros(1, dtype=torch.int32, device=dev)
    seen = torch.zeros(8, 3072, dtype=torch.uint8, device=dev)
    timed(lambda: K.sample(lg, 8, 3072, 3072, tok), "sample greedy V=3072")
    timed(lambda: K.sample(lg, 8, 3072, 3072, tok, seen=seen, rep_penalty=1.05, n_generated=step, min_new_tokens=2,
                           eos_id=2150, suppress=(2048, 3072, 2150)), "sample greedy + processors")
    timed(lambda: K.sample(lg, 8, 3072, 3072, tok, do_sample=True, top_k=50, temperature=0.9, step=step, seed=1),
          "sample top-k 50 V=3072")
    timed(lambda: K.sample(lg, 8, 3072, 3072, tok, do_sample=True, top_k=0, temperature=0.9, step=step, seed=1),
          "sample no-top-k V=3072")
    timed(lambda: K.sample(lg[:, :2048].contiguous(), 8, 2048, 2048, tok, do_sample=True, top_k=50, temperature=0.9,
                           step=step, seed=1), "sample top-k 50 V=2048")
    # decode attention
    for L in (17, 300, 460):
        B, Hq, Hkv, D = 8, 16, 8, 128
        qkv = torch.randn(B, (Hq + 2 * Hkv) * D, device=dev)
        kc = torch.randn(B, Hkv, L + 4, D, device=dev).bfloat16()
        vc = torch.randn(B, Hkv, L + 4, D, device=dev).bfloat16()
        qn = torch.ones(D, device=dev)
        cos, sin = K.rope_tables(D, 1e6, 4096, dev)
        i32 = lambda t: torch.as_tensor(t, dtype=torch.int32, device=dev)  # noqa: E731
        pos, rb, st = i32([L - 1] * B), i32(range(B)), i32([0] * B)
        out = torch.zeros(B, Hq * D, device=dev)
        for ns in ((1,) if L == 17 else (1, 2, 4)):
            ws = torch.zeros(K.decode_attn_ws_bytes(B, Hq, Hkv, D, ns), dtype=torch.uint8, device=dev)
            timed(lambda: K.decode_attention(qkv, B, Hq, Hkv, D, qn, qn, 1e-6, cos, sin, pos, rb, pos, st, kc, vc, L + 4,
                                             out, nsplit=ns, ws=ws), f"decode attention B=8 L={L} nsplit={ns}")


if __name__ == "__main__":
    main()
