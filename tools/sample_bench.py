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


if __name__ == "__main__":
    main()
