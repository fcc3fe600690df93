"""Code-predictor decode step at the 1.7B dims (B = 8, 17 keys), graph-captured, weights resident in the Infinity
Cache as in the frame: the launch-per-op chain (5 x {qkv GEMV (not layer 0), fused attention + o_proj, gate/up,
down} + lm_head = 20 launches) vs the persistent MLP form (5 x {fused attention + o_proj, qt_cp_mlp: gate/up ->
down -> next qkv | lm_head} + the tag-buffer clear = 11 launches)."""
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
    gu_w = [K.tile_swiglu(torch.randn(I, H, device=dev) * 0.02, torch.randn(I, H, device=dev) * 0.02, dt)
            for _ in range(nl)]
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
    tags = torch.zeros(K.cp_mlp_tags_bytes(H, I), dtype=torch.uint8, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    ctr = torch.zeros(1, dtype=torch.int32, device=dev)

    def attn(l):
        K.decode_attn_oproj(qkv, B, hq, hkv, D, qn, qn, 1e-6, cos, sin, kc[l], vc[l], L + 1, o_w[l], x,
                            const_pos=L - 1, x16=x16)

    def step_launches():
        for l in range(nl):
            if l:
                K.gemm(x16, qkv_w[l], qkv, B, H, (hq + 2 * hkv) * D, rms=True, eps=1e-6)
            attn(l)
            K.gemm(x16, gu_w[l], hmid, B, H, I, rms=True, eps=1e-6, epi=_hip.EPI_SWIGLU)
            K.gemm(hmid, dn_w[l], x, B, I, H, epi=_hip.EPI_ADD, out2=x16)
        K.gemm(x16, head, logits, B, H, V, rms=True, eps=1e-6)

    def step_persistent():
        tags.zero_()
        for l in range(nl):
            attn(l)
            w3, o3 = (qkv_w[l + 1], qkv) if l + 1 < nl else (head, logits)
            K.cp_mlp(x16, x, B, H, I, gu_w[l], dn_w[l], w3, o3, 1e-6, tags, ctr, l + 1, err)

    def mlp_only():
        for l in range(nl):
            w3, o3 = (qkv_w[l + 1], qkv) if l + 1 < nl else (head, logits)
            K.cp_mlp(x16, x, B, H, I, gu_w[l], dn_w[l], w3, o3, 1e-6, tags, ctr, l + 1, err)

    def gemv3_only():
        for l in range(nl):
            K.gemm(x16, gu_w[l], hmid, B, H, I, rms=True, eps=1e-6, epi=_hip.EPI_SWIGLU)
            K.gemm(hmid, dn_w[l], x, B, I, H, epi=_hip.EPI_ADD, out2=x16)
            w3 = qkv_w[l + 1] if l + 1 < nl else head
            K.gemm(x16, w3, qkv if l + 1 < nl else logits, B, H, w3.N, rms=True, eps=1e-6)

    if os.environ.get("QT_CPMLP_STOP"):  # phase timing: the MLP launches alone (the tag sequence restarts per replay:
        tags.zero_()                      # a stale tag only matches in the first run, so time the launches alone)
        microbench.timed(lambda: (tags.zero_(), mlp_only()), f"cp_mlp x5 + clear, stop={os.environ['QT_CPMLP_STOP']}")
        microbench.timed(gemv3_only, "three GEMVs x5")
        return
    microbench.N = 20
    for rep in range(2):
        a = microbench.timed(step_launches, f"[{rep}] CP step, launch per op (20 launches)")
        b = microbench.timed(step_persistent, f"[{rep}] CP step, persistent MLP (11 launches)")
        print(f"{'':60s} -> {a - b:6.2f} us saved per step, err {int(err.item())}", flush=True)


if __name__ == "__main__":
    main()
