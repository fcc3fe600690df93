"""Thin Python launchers over the C ABI (include/qwen3tts_amd.h) + weight re-layout helpers.

Every launcher takes torch device tensors (memory/plumbing only) and calls one `qt_*` entry point on
the current stream, so the calls are capturable into HIP graphs.
"""
from __future__ import annotations

import ctypes
import threading
from dataclasses import dataclass
from typing import Optional

import torch
import torch.nn.functional as F

from . import _hip
from ._hip import ptr, stream, check

KT_OF = {torch.bfloat16: 32, torch.float32: 16}


@dataclass
class Tiled:
    """A weight pre-tiled into MFMA B-fragment order (see csrc/gemm.hip)."""
    w: torch.Tensor
    N: int            # logical output width (rows of W; SwiGLU: 2*I)
    Np: int           # padded to 16
    K: int            # logical K (linear) or taps*cin (conv)
    Kp: int
    dtype: torch.dtype
    bias: Optional[torch.Tensor] = None
    taps: int = 0
    cin: int = 0
    cin_pad: int = 0


def tile(w: torch.Tensor, dtype: torch.dtype, bias=None, taps=0, cin=0, cin_pad=0, K=None) -> Tiled:
    """w: row-major [N][Kp'] on device (any float dtype) -> Tiled (N padded to 16, K padded to KT)."""
    kt = KT_OF[dtype]
    w = w.to(dtype)
    N, K0 = w.shape
    Kp = (K0 + kt - 1) // kt * kt
    if Kp != K0:
        w = F.pad(w, (0, Kp - K0))
    Np = (N + 15) // 16 * 16
    out = torch.empty(Np * Kp, dtype=dtype, device=w.device)
    w = w.contiguous()
    check(_hip.lib().qt_tile_weight(ptr(w), _hip.dtype_code(dtype), N, Kp, ptr(out), stream()), "qt_tile_weight")
    b = None
    if bias is not None:
        b = torch.zeros(Np, dtype=torch.float32, device=w.device)
        b[:N] = bias.float()
    return Tiled(out, N, Np, K if K is not None else K0, Kp, dtype, b, taps, cin, cin_pad)


def tile_linear(w, dtype, bias=None, gamma=None):
    """gamma: RMSNorm weight folded into the columns (W[n][k] * gamma[k]); use gemm(..., rms=True)."""
    if gamma is not None:
        w = w.float() * gamma.float()[None, :]
    return tile(w, dtype, bias)


def tile_swiglu(gate, up, dtype, gamma=None):
    """Interleave 8 gate rows / 8 up rows per 16-row tile (QT_EPI_SWIGLU pairing); optional folded RMSNorm gamma."""
    if gamma is not None:
        gate, up = gate.float() * gamma.float()[None, :], up.float() * gamma.float()[None, :]
    I, K = gate.shape
    assert I % 8 == 0
    w = torch.cat([gate.reshape(I // 8, 8, K), up.reshape(I // 8, 8, K)], 1).reshape(2 * I, K)
    return tile(w, dtype)


def _pad_cin(w, cin, dtype):
    kt = KT_OF[dtype]
    cp = (cin + kt - 1) // kt * kt
    return F.pad(w, (0, cp - cin)), cp


def tile_conv(w, b, dtype, dilation=1):
    """Causal Conv1d weight [Cout][Cin][k] -> implicit-GEMM layout [Cout][k][Cin_pad]."""
    cout, cin, k = w.shape
    wk, cp = _pad_cin(w.permute(0, 2, 1), cin, dtype)
    t = tile(wk.reshape(cout, k * cp), dtype, b, taps=k, cin=cin, cin_pad=cp, K=k * cp)
    t.dil = dilation
    return t


def tile_transconv(w, b, dtype, stride):
    """ConvTranspose1d weight [Cin][Cout][k] (k = 2*stride, trimmed by stride each side, K:195-207) as a
    2-tap 'valid' conv with stride*Cout outputs: out[(q-1)*s + r] = W[..., r+s]^T x[q-1] + W[..., r]^T x[q].
    k == stride (no trim): 1 tap, out[q*s + r] = W[..., r]^T x[q].  Channels-last output rows are then
    already in time order (pixel shuffle is free)."""
    cin, cout, k = w.shape
    s = stride
    if k == s:
        wr = w.permute(2, 1, 0).reshape(s * cout, 1, cin)  # [(r, co)][tap][ci]
        taps = 1
    else:
        assert k == 2 * s
        j0 = w[:, :, s:].permute(2, 1, 0)  # x[q-1] tap
        j1 = w[:, :, :s].permute(2, 1, 0)  # x[q]   tap
        wr = torch.stack([j0, j1], 2).reshape(s * cout, 2, cin)
        taps = 2
    wk, cp = _pad_cin(wr, cin, dtype)
    t = tile(wk.reshape(s * cout, taps * cp), dtype, b.repeat(s) if b is not None else None, taps=taps, cin=cin,
             cin_pad=cp, K=taps * cp)
    t.dil = 1
    return t


_WS = {}
# workspaces selected by `use_workspace`, a stack per host thread: two threads issuing on different streams each
# route their GEMMs through their own workspace (a module-global stack would hand one thread's ws to the other)
_TLS = threading.local()


def _active_stack():
    st = getattr(_TLS, "ws", None)
    if st is None:
        st = _TLS.ws = []
    return st


WS_BYTES = 16 << 20  # >= GEMM_WS_MIN: room for gemm_pf2_k's split-K records of the 17+-row linears


def new_workspace(device):
    """Split-K scratch of the decode GEMV and of gemm_pf2_k's narrow-output split-K (arrival counters must start at
    zero; every launch re-arms them).  One workspace per concurrently running stream."""
    return torch.zeros(max(WS_BYTES, _hip.GEMM_WS_MIN), dtype=torch.uint8, device=device)


def gemm_workspace(device):
    """Default per-device workspace, for single-stream callers.  Allocate before any graph capture."""
    idx = torch.device(device).index or 0
    if idx not in _WS:
        _WS[idx] = new_workspace(device)
    return _WS[idx]


_SIDE = {}


def side_stream(device):
    """A persistent side stream per device for work overlapped with the current stream (the voice-clone front ends,
    the reference-frame codec decode).  Persistent so its caching-allocator pool is reused: a fresh stream per call
    allocates fresh blocks, and hipMalloc stalls the host until the GPU is idle, which serialised the overlap."""
    idx = torch.device(device).index or 0
    if idx not in _SIDE:
        _SIDE[idx] = torch.cuda.Stream(device=device)
    return _SIDE[idx]


class use_workspace:
    """`with use_workspace(ws):` routes this host thread's qt_gemm calls (split-K records, im2col images) through
    `ws` -- one workspace per stream that can run concurrently (a session's, a codec stream slot's).  The selection
    is per host thread; without one the device's default workspace (single-stream callers) is used."""

    def __init__(self, ws):
        self.ws = ws

    def __enter__(self):
        _active_stack().append(self.ws)

    def __exit__(self, *exc):
        _active_stack().pop()


def active_workspace(device):
    st = _active_stack()
    return st[-1] if st else _WS.get(torch.device(device).index or 0)


def gemm(A, W: Tiled, out, M, lda, ldo, *, a_dtype=None, o_dtype=None, gamma=None, eps=0.0, rms=False, colscale=None,
         act=_hip.ACT_NONE, epi=_hip.EPI_STORE, a_index=None, conv=None, use_bias=True, splitk=0, snake=None,
         a_act=_hip.AACT_NONE, out2=None, ldo2=None):
    """conv = (t_in, t_out, t_off, dil) for implicit-conv weights.  splitk: 0 auto, 1 off, n forced
    (decode GEMV; 0 / 1 also for gemm_pf2_k's narrow-output split-K; needs gemm_workspace(device) allocated).  snake = (alpha, inv_beta): SnakeBeta applied
    to A per input channel inside the GEMM (fused codec activation).  out2: bf16 copy of the stored fp32 output
    (M <= 16; the decode residual stream's shadow read by the next RMS-normalised GEMV)."""
    a = _hip.GemmArgs()
    a.M, a.N, a.K = M, W.N, W.K
    a.a_dtype = _hip.dtype_code(a_dtype or A.dtype)
    a.w_dtype = _hip.dtype_code(W.dtype)
    a.o_dtype = _hip.dtype_code(o_dtype or out.dtype)
    a.A, a.lda, a.a_index = ptr(A), lda, ptr(a_index)
    a.W, a.gamma, a.eps, a.rmsnorm = ptr(W.w), ptr(gamma), eps, int(rms or gamma is not None)
    a.bias = ptr(W.bias) if use_bias else None
    a.colscale, a.act, a.epi = ptr(colscale), act, epi
    a.out, a.ldo = ptr(out), ldo
    if snake is not None:
        a.snake_alpha, a.snake_inv_beta = ptr(snake[0]), ptr(snake[1])
    a.a_act = a_act
    if out2 is not None:
        a.out2, a.ldo2 = ptr(out2), ldo if ldo2 is None else ldo2
    ws = active_workspace(out.device)
    if ws is not None:  # (convs: the short-window im2col route keeps its image in the workspace's upper half)
        a.ws, a.ws_bytes, a.splitk = ptr(ws), ws.numel(), splitk
    if W.taps:
        t_in, t_out, t_off, dil = conv
        a.taps, a.dil, a.cin, a.cin_pad, a.t_in, a.t_out, a.t_off = W.taps, dil, W.cin, W.cin_pad, t_in, t_out, t_off
    check(_hip.lib().qt_gemm(ctypes.byref(a), stream()), "qt_gemm")


def qkv_post(qkv, R, Hq, Hkv, D, q_norm, k_norm, eps, cos, sin, rope_pos, row_batch, kv_pos, q_out, kc, vc, Lmax):
    a = _hip.QkvArgs()
    a.R, a.Hq, a.Hkv, a.D = R, Hq, Hkv, D
    a.qkv, a.q_norm, a.k_norm, a.eps = ptr(qkv), ptr(q_norm), ptr(k_norm), eps
    a.cos_tab, a.sin_tab = ptr(cos), ptr(sin)
    a.rope_pos, a.row_batch, a.kv_pos = ptr(rope_pos), ptr(row_batch), ptr(kv_pos)
    a.q_out, a.k_cache, a.v_cache = ptr(q_out), ptr(kc), ptr(vc)
    a.kv_dtype, a.Lmax = _hip.dtype_code(kc.dtype), Lmax
    check(_hip.lib().qt_qkv_post(ctypes.byref(a), stream()), "qt_qkv_post")


def attention(q, R, Hq, Hkv, D, kc, vc, Lmax, row_batch, row_start, row_len, out, max_keys, window=0):
    a = _hip.AttnArgs()
    a.R, a.Hq, a.Hkv, a.D, a.Lmax, a.window = R, Hq, Hkv, D, Lmax, window
    a.q, a.k_cache, a.v_cache, a.kv_dtype = ptr(q), ptr(kc), ptr(vc), _hip.dtype_code(kc.dtype)
    a.row_batch, a.row_start, a.row_len = ptr(row_batch), ptr(row_start), ptr(row_len)
    a.out, a.o_dtype, a.max_keys = ptr(out), _hip.dtype_code(out.dtype), max_keys
    check(_hip.lib().qt_attention(ctypes.byref(a), stream()), "qt_attention")


def small_prefill_attention(qkv, R, T, Hq, Hkv, D, q_norm, k_norm, eps, cos, sin, kc, vc, Lmax, out):
    """qt_small_prefill_attention: rows b*T + t at positions t < T, keys all new (one launch)."""
    a = _hip.DecodeAttnArgs()
    a.R, a.Hq, a.Hkv, a.D, a.Lmax = R, Hq, Hkv, D, Lmax
    a.qkv, a.q_norm, a.k_norm, a.eps = ptr(qkv), ptr(q_norm), ptr(k_norm), eps
    a.cos_tab, a.sin_tab = ptr(cos), ptr(sin)
    a.k_cache, a.v_cache, a.kv_dtype = ptr(kc), ptr(vc), _hip.dtype_code(kc.dtype)
    a.out, a.o_dtype = ptr(out), _hip.dtype_code(out.dtype)
    check(_hip.lib().qt_small_prefill_attention(ctypes.byref(a), T, stream()), "qt_small_prefill_attention")


def decode_attn_ws_bytes(R, Hq, Hkv, D, nsplit):
    return int(_hip.lib().qt_decode_attn_ws_bytes(R, Hq, Hkv, D, nsplit))


def decode_attention(qkv, R, Hq, Hkv, D, q_norm, k_norm, eps, cos, sin, rope_pos, row_batch, kv_pos, row_start,
                     kc, vc, Lmax, out, window=0, const_pos=-1, nsplit=1, ws=None):
    """nsplit > 1: split-KV over nsplit blocks per (row, kv head); ws from decode_attn_ws_bytes (zeroed)."""
    a = _hip.DecodeAttnArgs()
    a.R, a.Hq, a.Hkv, a.D, a.Lmax, a.window = R, Hq, Hkv, D, Lmax, window
    a.qkv, a.q_norm, a.k_norm, a.eps = ptr(qkv), ptr(q_norm), ptr(k_norm), eps
    a.cos_tab, a.sin_tab = ptr(cos), ptr(sin)
    a.rope_pos, a.row_batch, a.kv_pos, a.row_start = ptr(rope_pos), ptr(row_batch), ptr(kv_pos), ptr(row_start)
    a.k_cache, a.v_cache, a.kv_dtype, a.out = ptr(kc), ptr(vc), _hip.dtype_code(kc.dtype), ptr(out)
    a.o_dtype = _hip.dtype_code(out.dtype)
    a.const_pos = const_pos
    a.nsplit = nsplit
    if ws is not None:
        a.ws, a.ws_bytes = ptr(ws), ws.numel() * ws.element_size()
    check(_hip.lib().qt_decode_attention(ctypes.byref(a), stream()), "qt_decode_attention")


def attn_oproj_ws_bytes(N, Hkv):
    return int(_hip.lib().qt_attn_oproj_ws_bytes(N, Hkv))


def decode_attn_oproj(qkv, R, Hq, Hkv, D, q_norm, k_norm, eps, cos, sin, kc, vc, Lmax, w_o: "Tiled", x, *,
                      const_pos=-1, rope_pos=None, kv_pos=None, row_start=None, x16=None, ws=None):
    """qt_decode_attn_oproj: x[:R] += o_proj(decode attention) in one launch (row r = batch entry r, short caches).
    x16: bf16 shadow of x, updated alongside.  ws: zeroed uint8 scratch of attn_oproj_ws_bytes(N, Hkv), private to
    one stream -- enables the head-split form (its int32 word 0 is the sticky hand-off error flag)."""
    a = _hip.AttnOprojArgs()
    a.R, a.Hq, a.Hkv, a.D, a.Lmax = R, Hq, Hkv, D, Lmax
    a.qkv, a.q_norm, a.k_norm, a.eps = ptr(qkv), ptr(q_norm), ptr(k_norm), eps
    a.cos_tab, a.sin_tab = ptr(cos), ptr(sin)
    a.rope_pos, a.kv_pos, a.row_start, a.const_pos = ptr(rope_pos), ptr(kv_pos), ptr(row_start), const_pos
    a.k_cache, a.v_cache, a.kv_dtype = ptr(kc), ptr(vc), _hip.dtype_code(kc.dtype)
    a.w_o, a.w_dtype, a.N = ptr(w_o.w), _hip.dtype_code(w_o.dtype), w_o.N
    a.x, a.ldx = ptr(x), x.stride(0)
    if x16 is not None:
        a.x16, a.ldx16 = ptr(x16), x16.stride(0)
    if ws is not None:
        a.ws, a.ws_bytes = ptr(ws), ws.numel() * ws.element_size()
    check(_hip.lib().qt_decode_attn_oproj(ctypes.byref(a), stream()), "qt_decode_attn_oproj")


def cp_step_ws_bytes():
    return int(_hip.lib().qt_cp_step_ws_bytes())


def cp_step_supported(H, I, Hq, Hkv, D, n_layers, V) -> bool:
    return bool(_hip.lib().qt_cp_step_supported(H, I, Hq, Hkv, D, n_layers, V))


def cp_step(layers, w_lm: "Tiled", x, qkv0, R, kcs, vcs, Lmax, const_pos, cos, sin, eps, logits, ws, sample=None):
    """qt_cp_step: one code-predictor decode step (every layer + final norm + lm_head) in one persistent launch.
    layers: the code predictor's _Layer objects (tiled qkv / o / gate-up / down, q_norm / k_norm); kcs / vcs: per-layer
    bf16 caches [R][Hkv][Lmax][D]; x fp32 [R][H] input rows; qkv0 fp32 [R][qkv] layer-0 q/k/v rows; logits fp32 [R][V].
    ws: zeroed uint8 scratch of cp_step_ws_bytes() kept across launches (word 0: the sticky hand-off error flag).
    sample: qt_sample_args (sample(..., launch=False), with emb and emb2 tables) of the PREVIOUS step's token choice:
    qt_cp_step_sampled runs it at the start of this launch and takes x / q/k/v from the chosen tokens' table rows."""
    a = _hip.CpStepArgs()
    a.R, a.n_layers, a.Lmax, a.const_pos, a.V, a.eps = R, len(layers), Lmax, const_pos, w_lm.N, eps
    a.cos_tab, a.sin_tab = ptr(cos), ptr(sin)
    for i, L in enumerate(layers):
        a.w_qkv[i], a.w_o[i], a.w_gu[i], a.w_down[i] = ptr(L.qkv.w), ptr(L.o.w), ptr(L.gu.w), ptr(L.down.w)
        a.q_norm[i], a.k_norm[i] = ptr(L.q_norm), ptr(L.k_norm)
        a.k_cache[i], a.v_cache[i] = ptr(kcs[i]), ptr(vcs[i])
    a.w_lm = ptr(w_lm.w)
    a.x, a.ldx = ptr(x), x.stride(0)
    a.qkv0, a.ldq = ptr(qkv0), qkv0.stride(0)
    a.logits, a.ldl = ptr(logits), logits.stride(0)
    a.ws, a.ws_bytes = ptr(ws), ws.numel() * ws.element_size()
    if sample is not None:
        check(_hip.lib().qt_cp_step_sampled(ctypes.byref(a), ctypes.byref(sample), stream()), "qt_cp_step_sampled")
        return
    check(_hip.lib().qt_cp_step(ctypes.byref(a), stream()), "qt_cp_step")


def cp_prefill(layers, w_lm: "Tiled", x, R, kcs, vcs, Lmax, cos, sin, eps, logits, ws):
    """qt_cp_prefill: the code predictor's 2-token prefill (positions 0, 1 of R batch rows: x fp32 [2R][H], rows 2b,
    2b + 1) through every layer + lm_head[0] for position 1 (logits [R][V]) in one launch of the step engine; the
    keys / values land at cache positions 0, 1.  Same workspace as cp_step."""
    a = _hip.CpStepArgs()
    a.R, a.n_layers, a.Lmax, a.const_pos, a.V, a.eps = R, len(layers), Lmax, 0, w_lm.N, eps
    a.cos_tab, a.sin_tab = ptr(cos), ptr(sin)
    for i, L in enumerate(layers):
        a.w_qkv[i], a.w_o[i], a.w_gu[i], a.w_down[i] = ptr(L.qkv.w), ptr(L.o.w), ptr(L.gu.w), ptr(L.down.w)
        a.q_norm[i], a.k_norm[i] = ptr(L.q_norm), ptr(L.k_norm)
        a.k_cache[i], a.v_cache[i] = ptr(kcs[i]), ptr(vcs[i])
    a.w_lm = ptr(w_lm.w)
    a.x, a.ldx = ptr(x), x.stride(0)
    a.logits, a.ldl = ptr(logits), logits.stride(0)
    a.ws, a.ws_bytes = ptr(ws), ws.numel() * ws.element_size()
    check(_hip.lib().qt_cp_prefill(ctypes.byref(a), stream()), "qt_cp_prefill")


def talker_tail_ws_bytes():
    return int(_hip.lib().qt_talker_tail_ws_bytes())


def talker_tail_supported(H, I, Hq, D, qkv_w) -> bool:
    return bool(_hip.lib().qt_talker_tail_supported(H, I, Hq, D, qkv_w))


def talker_tail(att, x, R, layer, next_layer, qkv, eps, ws):
    """qt_talker_tail: o_proj + residual -> gate/up + SwiGLU -> down + residual -> (next_layer given) its q/k/v rows, in
    one persistent launch.  att bf16 [R][Hq*D] attention rows; x fp32 [R][H] residual rows (updated in place); qkv fp32
    [R][qkv] out; layer / next_layer: the talker's _Layer objects.  ws: zeroed uint8 scratch of talker_tail_ws_bytes()
    kept across launches (word 0: the sticky hand-off error flag)."""
    a = _hip.TalkerTailArgs()
    a.R, a.eps = R, eps
    a.att, a.lda = ptr(att), att.stride(0)
    a.x, a.ldx = ptr(x), x.stride(0)
    a.w_o, a.w_gu, a.w_down = ptr(layer.o.w), ptr(layer.gu.w), ptr(layer.down.w)
    a.w_qkv_next = ptr(next_layer.qkv.w) if next_layer is not None else None
    a.qkv, a.ldq = (ptr(qkv), qkv.stride(0)) if next_layer is not None else (None, 0)
    a.ws, a.ws_bytes = ptr(ws), ws.numel() * ws.element_size()
    a.H, a.I = layer.o.N, layer.gu.N // 2  # the config's hidden / intermediate sizes (the engine is built for both talkers)
    check(_hip.lib().qt_talker_tail(ctypes.byref(a), stream()), "qt_talker_tail")


def sample(logits, R, V, ld, tok_out, *, seen=None, rep_penalty=1.0, n_generated=None, min_new_tokens=0, eos_id=-1,
           suppress=(0, 0, -1), ignore_eos=False, finished=None, do_sample=False, top_k=0, top_p=1.0,
           temperature=1.0, seed=0, step=None, substep=0, codes=None, codes_ld=0, codes_w=16, codes_col=0,
           codes_step_off=0, row_base=0, emb=None, seed_ptr=None, debug_u=-1.0, emb16=None, emb2=None, algo=0,
           ctr_stride=0, philox_row=None, force=None, pick=None, launch=True):
    """launch=False: return the qt_sample_args instead (for qt_cp_step_sampled).
    step / n_generated: device int32 counters, one per row when ctr_stride = 1 (0: shared); philox_row: optional
    device int32 [R] Philox stream ids (default row_base + r).
    force / pick (teacher forcing, parity diagnostics): int32 buffers in the layout of `codes`; the choice is stored
    in pick and the row continues with force's token.
    emb = (table fp32 [V][D], out fp32 rows, ld): also write the chosen token's table row to out[r];
    emb16 = (out bf16 rows, ld): its bf16 copy; emb2 = (table2 fp32 [V][D2], out2 fp32 rows, ld2): a second row.
    seed_ptr: device int64 [1] read at run time instead of `seed` (graph-captured samplers)."""
    a = _hip.SampleArgs()
    a.logits, a.R, a.V, a.ld = ptr(logits), R, V, ld
    a.seen, a.rep_penalty = ptr(seen), rep_penalty
    a.n_generated, a.min_new_tokens, a.eos_id = ptr(n_generated), min_new_tokens, eos_id
    a.suppress_lo, a.suppress_hi, a.suppress_keep = suppress
    a.ignore_eos, a.finished = int(ignore_eos), ptr(finished)
    a.do_sample, a.top_k, a.top_p, a.temperature = int(do_sample), int(top_k or 0), float(top_p), float(temperature)
    a.seed, a.step, a.substep, a.tok_out = seed & (2 ** 64 - 1), ptr(step), substep, ptr(tok_out)
    a.codes, a.codes_ld, a.codes_w, a.codes_col, a.codes_step_off = ptr(codes), codes_ld, codes_w, codes_col, codes_step_off
    a.row_base = row_base
    a.seed_ptr, a.debug_u, a.algo = ptr(seed_ptr), float(debug_u), int(algo)
    a.ctr_stride, a.philox_row = int(ctr_stride), ptr(philox_row)
    a.force, a.pick = ptr(force), ptr(pick)
    if emb is not None:
        a.emb_table, a.emb_dim, a.emb_out, a.emb_ld = ptr(emb[0]), emb[0].shape[1], ptr(emb[1]), emb[2]
        if emb16 is not None:
            a.emb_out16, a.emb_ld16 = ptr(emb16[0]), emb16[1]
        if emb2 is not None:
            a.emb2_table, a.emb2_dim, a.emb2_out, a.emb2_ld = ptr(emb2[0]), emb2[0].shape[1], ptr(emb2[1]), emb2[2]
    if not launch:
        return a
    check(_hip.lib().qt_sample(ctypes.byref(a), stream()), "qt_sample")


def rmsnorm(x, g, eps, out, M, N, rec=None, step=None, step_off=0, step_stride=0):
    """rec: also store the rows at rec[m, step[m * step_stride] + step_off] (rec [M][F][N] fp32, step device int32
    counters: one shared (stride 0) or one per row)."""
    if rec is None:
        check(_hip.lib().qt_rmsnorm(ptr(x), ptr(g), eps, ptr(out), M, N, stream()), "qt_rmsnorm")
    else:
        check(_hip.lib().qt_rmsnorm_rec(ptr(x), ptr(g), eps, ptr(out), M, N, ptr(rec), rec.stride(0), ptr(step),
                                        step_off, step_stride, stream()), "qt_rmsnorm_rec")


def gather_rows(table, idx, M, H, out, ldo):
    check(_hip.lib().qt_gather_rows(ptr(table), _hip.dtype_code(table.dtype), ptr(idx), M, H, ptr(out), ldo, stream()),
          "qt_gather_rows")


def frame_embed(e0, ecp, G, H, codes, codes_ld, step, trailing, T, pad, x, B, x16=None, step_stride=0):
    check(_hip.lib().qt_frame_embed(ptr(e0), ptr(ecp), _hip.dtype_code(e0.dtype), e0.shape[0], ecp.shape[1], G, H,
                                    ptr(codes), codes_ld, ptr(step), step_stride, ptr(trailing), T, ptr(pad), ptr(x),
                                    ptr(x16), B,
                                    stream()),
          "qt_frame_embed")


def advance(counters, n):
    check(_hip.lib().qt_advance(ptr(counters), n, stream()), "qt_advance")


def advance_rows(counters, B, nfields, cap):
    """Per-row counters [nfields][B] (field 0 = frame index): rows below cap advance every field by one."""
    check(_hip.lib().qt_advance_rows(ptr(counters), B, nfields, cap, stream()), "qt_advance_rows")


def rvq_gather(tables, Q, n_first, cb, dim, codes, B, T, o1, o2):
    check(_hip.lib().qt_rvq_gather(ptr(tables), Q, n_first, cb, dim, ptr(codes), B, T, ptr(o1), ptr(o2), stream()),
          "qt_rvq_gather")


def snake(x, y, rows, C, alpha, inv_beta):
    check(_hip.lib().qt_snake(ptr(x), ptr(y), _hip.dtype_code(x.dtype), rows, C, ptr(alpha), ptr(inv_beta), stream()),
          "qt_snake")


def dwconv_ln(x, B, T, C, w, b, lw, lb, eps, out):
    check(_hip.lib().qt_dwconv_ln(ptr(x), _hip.dtype_code(x.dtype), B, T, C, ptr(w), ptr(b), ptr(lw), ptr(lb), eps,
                                  ptr(out), stream()), "qt_dwconv_ln")


def clamp_pcm(x, n, out):
    check(_hip.lib().qt_clamp_pcm(ptr(x), _hip.dtype_code(x.dtype), n, ptr(out), stream()), "qt_clamp_pcm")


def rope_tables(head_dim: int, theta: float, npos: int, device):
    """cos/sin [npos][D/2] computed exactly as the reference (fp32 on CPU, M:526-592), then uploaded."""
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.int64).to(dtype=torch.float) / head_dim))
    f = torch.arange(npos, dtype=torch.float32)[:, None] * inv[None, :]
    return f.cos().contiguous().to(device), f.sin().contiguous().to(device)


# ---- voice-clone front end (csrc/frontend.hip) ----
def pad_time(x, B, T, C, left, right, mode, out, t_total=None, x2=None, ldx=None, ldx2=None, ldo=None):
    t_total = T + left + right if t_total is None else t_total
    check(_hip.lib().qt_pad_time(ptr(x), ldx or C, ptr(x2), ldx2 or C, _hip.dtype_code(x.dtype), B, T, C, left, right,
                                 mode, t_total, ptr(out), ldo or C, stream()), "qt_pad_time")


def zero_tail(x, B, Tp, v, C, ldx=None):
    check(_hip.lib().qt_zero_tail(ptr(x), _hip.dtype_code(x.dtype), B, Tp, v, C, ldx or C, stream()), "qt_zero_tail")


def layernorm(x, w, b, eps, out, M, N, ldx=None, ldo=None):
    check(_hip.lib().qt_layernorm(ptr(x), ldx or N, ptr(w), ptr(b), eps, ptr(out), _hip.dtype_code(out.dtype),
                                  ldo or N, M, N, stream()), "qt_layernorm")


def rvq_encode(x, ldx, tab, tabT, Q, cb, D, R, codes, codes_ld, ws=None):
    """ws: zero-initialised uint8 device scratch (reusable; allocated here when None)."""
    need = int(_hip.lib().qt_rvq_encode_ws_bytes(R, D, cb))
    if ws is None or ws.numel() < need:
        ws = torch.zeros(max(need, 1), dtype=torch.uint8, device=x.device)
    check(_hip.lib().qt_rvq_encode(ptr(x), ldx, ptr(tab), ptr(tabT), Q, cb, D, R, ptr(codes), codes_ld, ptr(ws),
                                   ws.numel(), stream()), "qt_rvq_encode")


def mel_logmag(spec, ld_spec, F_, nbin, basis, nmel, out, ldo=None):
    check(_hip.lib().qt_mel_logmag(ptr(spec), ld_spec, F_, nbin, ptr(basis), nmel, ptr(out), ldo or nmel, stream()),
          "qt_mel_logmag")


def time_stats(x, B, T, C, mean_out, std_out=None, logits=None, eps=1e-12, ldx=None, ldl=None, ld_out=None):
    check(_hip.lib().qt_time_stats(ptr(x), _hip.dtype_code(x.dtype), ldx or C, ptr(logits), ldl or C, B, T, C, eps,
                                   ptr(mean_out), ptr(std_out), ld_out or C, stream()), "qt_time_stats")


def scale_add(x, s, res, B, T, C, out, ldx=None, lds=None, ldr=None, ldo=None):
    check(_hip.lib().qt_scale_add(ptr(x), ldx or C, ptr(s), lds or C, ptr(res), ldr or C, _hip.dtype_code(x.dtype),
                                  B, T, C, ptr(out), ldo or C, stream()), "qt_scale_add")


def bcast_rows(v, B, T, W, out, ldv=None, ldo=None):
    check(_hip.lib().qt_bcast_rows(ptr(v), ldv or W, B, T, W, ptr(out), _hip.dtype_code(out.dtype), ldo or W, stream()),
          "qt_bcast_rows")
