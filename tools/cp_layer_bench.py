"""Code-predictor decode layer pieces at the 1.7B dims (B = 8, 17 keys): qkv GEMV, decode attention, o_proj GEMV
and the fused attention + o_proj (qt_decode_attn_oproj), alone and as dependent chains; graphs of N launches."""
import os
import sys
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "qwen3-tts_amd"))
from qwen_tts import kernels as K, _hip  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from microbench import timed  # noqa: E402

dev = torch.device("cuda:0")


def main():
    B, H, hq, hkv, D, L = 8, 1024, 16, 8, 128, int(os.environ.get("QT_CPL_KEYS", "17"))
    dt = torch.bfloat16
    K.gemm_workspace(dev)
    nl = 5
    qkv_w = [K.tile_linear(torch.randn((hq + 2 * hkv) * D, H, device=dev) * 0.02, dt) for _ in range(nl)]
    o_w = [K.tile_linear(torch.randn(H, hq * D, device=dev) * 0.02, dt) for _ in range(nl)]
    x = torch.randn(B, H, device=dev)
    qkv = torch.randn(B, (hq + 2 * hkv) * D, device=dev)
    qn = torch.ones(D, device=dev)
    kc = [torch.randn(B, hkv, L + 1, D, device=dev).to(dt) for _ in range(nl)]
    vc = [torch.randn(B, hkv, L + 1, D, device=dev).to(dt) for _ in range(nl)]
    cos, sin = K.rope_tables(D, 1e6, 64, dev)
    att = torch.zeros(B, hq * D, device=dev, dtype=dt)
    i32 = lambda t: torch.as_tensor(t, dtype=torch.int32, device=dev)  # noqa: E731
    pos, rb, zero = i32([L - 1] * B), i32(range(B)), i32([0] * B)
    it = {"i": 0}

    def nxt():
        it["i"] += 1
        return it["i"] % nl

    def qkv_gemv():
        K.gemm(x, qkv_w[nxt()], qkv, B, H, (hq + 2 * hkv) * D, rms=True, eps=1e-6)

    def attn():
        i = nxt()
        K.decode_attention(qkv, B, hq, hkv, D, qn, qn, 1e-6, cos, sin, pos, rb, pos, zero, kc[i], vc[i], L + 1, att,
                           const_pos=L - 1)

    def oproj():
        K.gemm(att, o_w[nxt()], x, B, hq * D, H, epi=_hip.EPI_ADD)

    def fused():
        i = nxt()
        K.decode_attn_oproj(qkv, B, hq, hkv, D, qn, qn, 1e-6, cos, sin, kc[i], vc[i], L + 1, o_w[i], x,
                            const_pos=L - 1)
    ws = torch.zeros(K.attn_oproj_ws_bytes(H, hkv), dtype=torch.uint8, device=dev)

    def fused_hs():
        i = nxt()
        K.decode_attn_oproj(qkv, B, hq, hkv, D, qn, qn, 1e-6, cos, sin, kc[i], vc[i], L + 1, o_w[i], x,
                            const_pos=L - 1, ws=ws)
    timed(qkv_gemv, "qkv GEMV 1024->4096 rms")
    timed(attn, "decode attention (17 keys)")
    timed(oproj, "o_proj GEMV 2048->1024 +res")
    timed(fused, "fused attention + o_proj")
    timed(fused_hs, "fused attention + o_proj, head-split (hand-offs)")

    def chain2():
        qkv_gemv(); attn(); oproj()

    def chain1():
        qkv_gemv(); fused()

    def chain1h():
        qkv_gemv(); fused_hs()
    timed(chain2, "chain qkv -> attn -> o_proj (per 3 launches)")
    timed(chain1, "chain qkv -> fused (per 2 launches)")
    timed(chain1h, "chain qkv -> fused head-split (per 2 launches)")
    print("hand-off error flag", int(ws[:4].view(torch.int32).item()))


if __name__ == "__main__":
    main()
