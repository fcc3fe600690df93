# Needs profiles/r02_l2_next_hint.diff applied (the hint was measured and not kept: profiles/r02_l2_next_hint_ab.txt).
"""L2 warm-up hint (qt_gemm_args.l2_next) on the code predictor's decode chain at the 1.7B dims (B = 8, 17 keys):
five layers of qkv GEMV -> fused attention + o_proj -> gate-up GEMV -> down GEMV (+ lm_head), weights resident in
the Infinity Cache as in the frame; each launch warms the next launch's weights into the L2 of the XCD that will
read them.  Graphs of N chained steps, hint on vs off, same process."""
import os
import sys
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "qwen3-tts_amd"))
from qwen_tts import kernels as K, _hip  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import microbench  # noqa: E402

dev = torch.device("cuda:0")


def main():
    B, H, hq, hkv, D, L, I, V = 8, 1024, 16, 8, 128, 17, 3072, 2048
    dt = torch.bfloat16
    K.gemm_workspace(dev)
    nl = 5
    rnd = lambda n, k: K.tile_linear(torch.randn(n, k, device=dev) * 0.02, dt)  # noqa: E731
    qkv_w = [rnd((hq + 2 * hkv) * D, H) for _ in range(nl)]
    o_w = [rnd(H, hq * D) for _ in range(nl)]
    gu_w = [rnd(2 * I, H) for _ in range(nl)]
    dn_w = [rnd(H, I) for _ in range(nl)]
    head = rnd(V, H)
    x = torch.randn(B, H, device=dev)
    x16 = x.to(dt)
    qkv = torch.randn(B, (hq + 2 * hkv) * D, device=dev)
    hmid = torch.zeros(B, I, device=dev, dtype=dt)
    logits = torch.zeros(B, V, device=dev)
    qn = torch.ones(D, device=dev)
    kc = [torch.randn(B, hkv, L + 1, D, device=dev).to(dt) for _ in range(nl)]
    vc = [torch.randn(B, hkv, L + 1, D, device=dev).to(dt) for _ in range(nl)]
    cos, sin = K.rope_tables(D, 1e6, 64, dev)

    def step(hint, decoy=False, only=("q", "a", "g", "d", "h")):
        # decoy: warm a different layer's weights of the same shapes (the warm-up's cost without its benefit)
        wl = (lambda l: (l + 2) % nl) if decoy else (lambda l: l)
        for l0 in range(nl):
            l = l0
            nxt_q = K.l2_gemv(qkv_w[wl(l + 1)]) if l + 1 < nl else K.l2_gemv(head)
            K.gemm(x16, qkv_w[l], qkv, B, H, (hq + 2 * hkv) * D, rms=True, eps=1e-6,
                   l2_next=K.l2_oproj(o_w[wl(l)]) if hint and "q" in only else None)
            K.decode_attn_oproj(qkv, B, hq, hkv, D, qn, qn, 1e-6, cos, sin, kc[l], vc[l], L + 1, o_w[l], x,
                                const_pos=L - 1, x16=x16, l2_next=K.l2_gemv(gu_w[wl(l)]) if hint and "a" in only else None)
            K.gemm(x16, gu_w[l], hmid, B, H, I, rms=True, eps=1e-6, epi=_hip.EPI_SWIGLU,
                   l2_next=K.l2_gemv(dn_w[wl(l)]) if hint and "g" in only else None)
            K.gemm(hmid, dn_w[l], x, B, I, H, epi=_hip.EPI_ADD, out2=x16, l2_next=nxt_q if hint and "d" in only else None)
        K.gemm(x16, head, logits, B, H, V, rms=True, eps=1e-6, l2_next=K.l2_gemv(qkv_w[0]) if hint and "h" in only else None)

    microbench.N = 20
    for rep in range(2):
        for hint, decoy, only in ((False, False, ""), (True, False, "qaghd"), (True, True, "qaghd"), (True, False, "a"),
                                  (True, True, "a"), (True, False, "q"), (True, False, "g"), (True, False, "d")):
            us = microbench.timed(lambda: step(hint, decoy, only),
                                  f"[{rep}] CP step, L2 hint {'decoy' if decoy else ('on' if hint else 'off')} [{only}]")
            print(f"{'':60s} -> {us / 21:8.2f} us per launch", flush=True)


if __name__ == "__main__":
    main()
