"""qt_sample latency at the code-predictor shape (R = 8, V = 2048, top-k 50, T 0.9, next-step embedding row) and
the talker shape (V = 3072 + processors); graphs of N launches.  QT_SAMPLE_STOP=n ends the kernel after phase n."""
import os
import sys
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "qwen3-tts_amd"))
from qwen_tts import kernels as K  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from microbench import timed  # noqa: E402

dev = torch.device("cuda:0")


def main():
    g = torch.Generator(device="cpu").manual_seed(0)
    lg = (torch.randn(8, 2048, generator=g) * 3).to(dev)
    tok = torch.zeros(8, dtype=torch.int32, device=dev)
    step = torch.zeros(1, dtype=torch.int32, device=dev)
    tab = torch.randn(2048, 1024, device=dev)
    out = torch.zeros(16, 1024, device=dev)
    tag = os.environ.get("QT_SAMPLE_STOP", "0")
    timed(lambda: K.sample(lg, 8, 2048, 2048, tok, do_sample=True, top_k=50, temperature=0.9, step=step, seed=1,
                           emb=(tab, out, 1024)), f"[stop={tag}] CP sample top-k 50 V=2048 + emb row")
    timed(lambda: K.sample(lg, 8, 2048, 2048, tok, do_sample=True, top_k=50, temperature=0.9, step=step, seed=1),
          f"[stop={tag}] CP sample top-k 50 V=2048")
    timed(lambda: K.sample(lg, 8, 2048, 2048, tok), f"[stop={tag}] greedy V=2048")
    # as in the frame: logits at the synthetic-weight scale (lm_head rows N(0, 0.02) x 1024 normalised inputs ->
    # std ~0.64), the bf16 shadow row, and the layer-0 q/k/v row gathered from 14 cold 2048 x 4096 fp32 tables
    lg2 = (torch.randn(8, 2048, generator=g) * 0.64).to(dev)
    o16 = torch.zeros(16, 1024, dtype=torch.bfloat16, device=dev)
    tabs = [torch.randn(2048, 4096, device=dev) for _ in range(14)]
    o2 = torch.zeros(16, 4096, device=dev)
    for algo in (0, 1):
        timed(lambda: K.sample(lg2, 8, 2048, 2048, tok, do_sample=True, top_k=50, temperature=0.9, step=step, seed=1,
                               emb=(tab, out, 1024), algo=algo), f"[algo={algo}] logits std 0.64 + emb row")
        it = {"i": 0}

        def f():
            K.sample(lg2, 8, 2048, 2048, tok, do_sample=True, top_k=50, temperature=0.9, step=step, seed=1,
                     emb=(tab, out, 1024), emb16=(o16, 1024), emb2=(tabs[it["i"] % 14], o2, 4096), algo=algo)
            it["i"] += 1
        timed(f, f"[algo={algo}] std 0.64 + emb + emb16 + cold emb2 (14 x 33.5 MB)")
    # the frame's pair: lm_head GEMV (bf16 shadow A, RMS folded) writing the logits, then the sampler reading them
    heads = [K.tile_linear(torch.randn(2048, 1024, device=dev) * 0.02, torch.bfloat16) for _ in range(15)]
    x16 = torch.randn(8, 1024, device=dev).to(torch.bfloat16)
    itc = {"i": 0}

    def head():
        K.gemm(x16, heads[itc["i"] % 15], lg2, 8, 1024, 2048, rms=True, eps=1e-6)
        itc["i"] += 1

    def pair():
        head()
        K.sample(lg2, 8, 2048, 2048, tok, do_sample=True, top_k=50, temperature=0.9, step=step, seed=1,
                 emb=(tab, out, 1024), emb16=(o16, 1024), emb2=(tabs[itc["i"] % 14], o2, 4096))
    timed(head, "lm_head GEMV alone")
    timed(pair, "lm_head GEMV + sampler (fresh logits)")


if __name__ == "__main__":
    main()
