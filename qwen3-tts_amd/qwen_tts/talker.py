"""MI355X talker + code-predictor engine: prompt assembly, prefill, graph-captured per-frame decode.

Replaces `Qwen3TTSForConditionalGeneration.generate` (M = qwen_tts/core/models/modeling_qwen3_tts.py,
:2022-2292) including the nested transformers-4.57 GenerationMixin loops of the talker (:2272) and the
code predictor (:1671-1680).  One frame = 15 code-predictor steps + one talker decode step + token
choice, captured once into a HIP graph and replayed per 80 ms frame; every step-dependent quantity
(positions, KV lengths, frame index) lives in device counters advanced by `qt_advance` inside the graph.
Per-request state lives in a `Session` object, never on the module (fixes the reference's shared
`rope_deltas` race).
"""
from __future__ import annotations

from collections import OrderedDict
from dataclasses import dataclass
from typing import Dict, List, Optional

import torch

from . import _hip
from . import kernels as K


def _to_dev_i32(ids, dev) -> torch.Tensor:
    """Token ids (list / host tensor / device tensor) as a flat device int32 tensor. Host ids go through pinned
    memory with a non-blocking copy: a pageable upload waits for all queued GPU work."""
    if isinstance(ids, torch.Tensor) and ids.device.type != "cpu":
        return ids.reshape(-1).to(dev, torch.int32)
    h = torch.as_tensor(ids, dtype=torch.int32).reshape(-1)
    if dev.type != "cuda":
        return h.to(dev)
    return h.pin_memory().to(dev, non_blocking=True)


def _w(W, name, dev):
    t = W[name]
    if not isinstance(t, torch.Tensor):
        t = torch.from_numpy(t)
    return t.to(dev)


class _Layer:
    def __init__(self, W, pre, lc, wdt, dev):
        g = lambda n: _w(W, f"{pre}.{n}", dev)  # noqa: E731
        # RMSNorm weights are folded into the following projection (W[n][k] * gamma[k]); the GEMM applies
        # the per-row rsqrt(mean(x^2) + eps) itself (rms=True)
        self.qkv = K.tile_linear(torch.cat([g("self_attn.q_proj.weight"), g("self_attn.k_proj.weight"),
                                            g("self_attn.v_proj.weight")], 0), wdt, gamma=g("input_layernorm.weight"))
        self.o = K.tile_linear(g("self_attn.o_proj.weight"), wdt)
        self.gu = K.tile_swiglu(g("mlp.gate_proj.weight"), g("mlp.up_proj.weight"), wdt,
                                gamma=g("post_attention_layernorm.weight"))
        self.down = K.tile_linear(g("mlp.down_proj.weight"), wdt)
        self.in_ln = g("input_layernorm.weight").float().contiguous()
        self.post_ln = g("post_attention_layernorm.weight").float().contiguous()
        self.q_norm = g("self_attn.q_norm.weight").float().contiguous()
        self.k_norm = g("self_attn.k_norm.weight").float().contiguous()


class _Stack:
    """One Qwen3 decoder stack (talker backbone or code predictor)."""

    def __init__(self, W, prefix, lc, wdt, dev, npos):
        self.H, self.I = lc["hidden_size"], lc["intermediate_size"]
        self.Hq, self.Hkv, self.D = lc["num_attention_heads"], lc["num_key_value_heads"], lc["head_dim"]
        self.eps = lc["rms_norm_eps"]
        self.n_layers = lc["num_hidden_layers"]
        self.layers = [_Layer(W, f"{prefix}.layers.{i}", lc, wdt, dev) for i in range(self.n_layers)]
        self.norm = _w(W, f"{prefix}.norm.weight", dev).float().contiguous()
        self.theta = lc["rope_theta"]
        self.cos, self.sin = K.rope_tables(self.D, self.theta, npos, dev)
        self.qkv_w = (self.Hq + 2 * self.Hkv) * self.D
        self.wdt = wdt

    def ensure_rope(self, npos, dev):
        """Grow the RoPE tables to >= npos positions.  The old tables stay alive: graphs captured by other sessions
        (frame / prefill graphs of pooled sessions) keep reading them, and they hold the same values."""
        if self.cos.shape[0] < npos:
            self._old_rope = getattr(self, "_old_rope", []) + [(self.cos, self.sin)]
            self.cos, self.sin = K.rope_tables(self.D, self.theta, max(npos, 2 * self.cos.shape[0]), dev)

    def forward(self, x, R, meta, kv, scratch, Lmax, max_keys, decode=False, x16=None, qkv0=False):
        """x fp32 [R][H] residual stream, updated in place.  meta: dict of int32 device row arrays.
        decode=True: one row per batch entry attending to its own prefix -> fused qt_decode_attention.
        x16 (bf16 mode, R <= 16): bf16 shadow of x, kept current by every writer of x (the residual-add epilogues
        store both) and read as the A operand of the RMS-normalised GEMVs (QKV, gate/up): their MFMA rounds A to
        bf16 anyway, so only the RMS row sums change (they come from the bf16 values, as the reference's bf16
        residual stream gives them) while the activation fetch halves.
        qkv0: scratch["qkv"] already holds layer 0's q/k/v rows (gathered by the previous step's sampler)."""
        # code-predictor decode steps: attention + o_proj + residual in one launch (qt_decode_attn_oproj)
        fused_ao = decode and scratch.get("attn_oproj", False) and meta.get("const_pos", -1) >= 0
        # talker decode: everything after each layer's attention in one launch (qt_talker_tail), which also computes
        # the next layer's q/k/v rows; the layer outputs go to x only (the bf16 shadow is not kept current)
        tail = decode and not fused_ao and scratch.get("tt_ws") is not None
        if x16 is not None and R > 96 and not PF:
            x16 = None  # igemm_k writes x only (decode / skinny GEMVs and gemm_pf_k keep the shadow)
        xa = x if x16 is None else x16
        for li, L in enumerate(self.layers):
            kc, vc = kv[0][li], kv[1][li]
            if not (qkv0 and li == 0) and not (tail and li > 0):
                K.gemm(xa, L.qkv, scratch["qkv"], R, self.H, self.qkv_w, rms=True, eps=self.eps)
            if fused_ao:
                K.decode_attn_oproj(scratch["qkv"], R, self.Hq, self.Hkv, self.D, L.q_norm, L.k_norm, self.eps,
                                    self.cos, self.sin, kc, vc, Lmax, L.o, x, const_pos=meta["const_pos"], x16=x16,
                                    ws=scratch.get("ao_ws"))
            elif decode:
                ns = meta.get("nsplit", 1)
                K.decode_attention(scratch["qkv"], R, self.Hq, self.Hkv, self.D, L.q_norm, L.k_norm, self.eps,
                                   self.cos, self.sin, meta["rope_pos"], meta["row_batch"], meta["kv_pos"],
                                   meta["row_start"], kc, vc, Lmax, scratch["att"], const_pos=meta.get("const_pos", -1),
                                   nsplit=ns, ws=scratch.get("attn_ws") if ns > 1 else None)
            elif "small_T" in meta:  # every key is new and rows are [batch][token]: one fused launch
                K.small_prefill_attention(scratch["qkv"], R, meta["small_T"], self.Hq, self.Hkv, self.D, L.q_norm,
                                          L.k_norm, self.eps, self.cos, self.sin, kc, vc, Lmax, scratch["att"])
            else:
                K.qkv_post(scratch["qkv"], R, self.Hq, self.Hkv, self.D, L.q_norm, L.k_norm, self.eps, self.cos,
                           self.sin, meta["rope_pos"], meta["row_batch"], meta["kv_pos"], scratch["q"], kc, vc, Lmax)
                K.attention(scratch["q"], R, self.Hq, self.Hkv, self.D, kc, vc, Lmax, meta["row_batch"],
                            meta["row_start"], meta["row_len"], scratch["att"], max_keys)
            if tail:
                nxt = self.layers[li + 1] if li + 1 < self.n_layers else None
                K.talker_tail(scratch["att"], x, R, L, nxt, scratch["qkv"], self.eps, scratch["tt_ws"])
                continue
            if not fused_ao:
                K.gemm(scratch["att"], L.o, x, R, self.Hq * self.D, self.H, epi=_hip.EPI_ADD, out2=x16)
            K.gemm(xa, L.gu, scratch["h"], R, self.H, self.I, rms=True, eps=self.eps, epi=_hip.EPI_SWIGLU)
            K.gemm(scratch["h"], L.down, x, R, self.I, self.H, epi=_hip.EPI_ADD, out2=x16)


# code-predictor decode steps: qt_decode_attn_oproj (attention fused into o_proj + residual); QT_ATTN_OPROJ=0 keeps
# the two-launch path (decode attention, then the o_proj GEMV) for A/B measurement
ATTN_OPROJ = _hip.lib_knob("QT_ATTN_OPROJ", 1) != 0
# ... for lanes of at most this many rows: every block of the fused kernel re-reads its o_proj weight slice per row
# (R x 4 MiB through L2 per launch), so at 64 rows it took 50.5 us per launch (bench --workload vd64 profile).
# vd64 audio-s/s with 16 / 32 / 64 refilled rows: fused 238 / 285 / 328, two launches 254 / 337 / 452
# (profiles/r03_attn_oproj_rows_ab.txt); at 8 rows the fused launch wins (round 2: 155.9 -> 164.0).  QT_ATTN_OPROJ_MAX
# overrides (A/B)
ATTN_OPROJ_MAX = _hip.lib_knob("QT_ATTN_OPROJ_MAX", 8)
# ... in its head-split form (qt_attn_oproj_args.ws: per-(column group, kv head) blocks exchanging row partials): 2.5x
# less L2 -> CU traffic than the (column group, row) form (profiles/r04_pmc_attn_oproj*.json), 7.71 -> 7.03 us per
# launch, bench 200.2 -> 202.8 audio-s/s (profiles/r04_bench_ab_ao_hs.txt).  QT_AO_HS=0 keeps the other form (A/B)
AO_HS = _hip.lib_knob("QT_AO_HS", 1) != 0
# code-predictor decode steps as ONE persistent launch each (qt_cp_step: every layer + lm_head, in-launch hand-offs)
# instead of ~21 dependent launches (bf16 mode with the layer-0 q/k/v tables, <= 8 rows); QT_CP_ENGINE=0 keeps the
# launch chain (A/B)
CP_ENGINE = _hip.lib_knob("QT_CP_ENGINE", 1) != 0
# ... and the per-frame 2-token prefill through the same engine (qt_cp_prefill: 16 token rows, one launch instead of
# ~26); QT_CP_PREFILL=0 keeps the launch chain for the prefill (A/B)
CP_PREFILL = _hip.lib_knob("QT_CP_PREFILL", 1) != 0
# ... and each step's token choice at the start of the NEXT step's launch (qt_cp_step_sampled: qt_sample's body on 4
# waves of 8 workgroups, the chosen rows handed to the rest in-launch) instead of its own launch; QT_CP_FUSE_SAMPLE=0
# keeps the qt_sample launches (A/B)
CP_FUSE_SAMPLE = _hip.lib_knob("QT_CP_FUSE_SAMPLE", 1) != 0
# talker decode layers: o_proj -> gate/up -> down -> next layer's q/k/v as ONE persistent launch per layer (qt_talker_tail:
# weights streamed through an LDS ring by loader waves, in-launch hand-offs) after each layer's attention, instead of
# four GEMV launches (bf16 mode, <= 8 rows, the 1.7B talker's shapes); QT_TALKER_TAIL=0 keeps the launch chain (A/B)
TALKER_TAIL = _hip.lib_knob("QT_TALKER_TAIL", 1) != 0
# bf16 residual shadows as the RMS-normalised GEMVs' A operand (bf16 mode); QT_X16=0 reads the fp32 stream (A/B)
X16 = _hip.lib_knob("QT_X16", 1) != 0
# code-predictor layer-0 q/k/v rows gathered from precomputed tables (bf16 mode); QT_QKV0_TAB=0 keeps the GEMV (A/B)
QKV0_TAB = _hip.lib_knob("QT_QKV0_TAB", 1) != 0
# talker prefill captured into a HIP graph per (session, prompt length) once that length repeats; QT_PREFILL_GRAPH=0
# always issues it eagerly (A/B)
PREFILL_GRAPH = _hip.lib_knob("QT_PREFILL_GRAPH", 1) != 0
# large-M prefill linears on gemm_pf_k (LDS-staged bf16 A and B): the prefill keeps the bf16 residual shadow at any
# row count, so its RMS GEMMs read bf16 A too; QT_PF=0 (read by the library as well) keeps igemm_k (A/B)
PF = _hip.lib_knob("QT_PF", 1) != 0  # as the library reads it (probe builds only)
# static prefill buffers (+ captured graphs) kept per session: the most recently used prompt lengths, LRU-evicted
PREFILL_CACHE = max(1, _hip.lib_knob("QT_PREFILL_CACHE", 4))
# the generation config's min_new_tokens (M:2044-2066): EOS is suppressed while a row has generated fewer tokens
MIN_NEW_TOKENS = 2
# talker decode attention split-KV by cache length: (keys below which, nsplit).  B = 8, 1.7B (tools/talker_attn_bench.py,
# profiles/r04_attn_long.txt, us per launch for nsplit 1 / 2 / 4 / 8): 512 keys 11.1 / 11.4 / 12.5 / 19.2, 1024 16.5 /
# 14.4 / 15.1 / 21.0, 2048 26.9 / 20.3 / 20.3 / 25.8, 4000 47.2 / 31.9 / 30.4 / 36.0.  The frame graph is captured once
# per split factor and the host picks the graph from its bound on the longest row's key count.  QT_ATTN_SPLIT=0 keeps
# one block per (row, kv head) at every length (A/B)
ATTN_SPLIT = [(768, 1), (2048, 2), (1 << 30, 4)] if _hip.lib_knob("QT_ATTN_SPLIT", 1) else [(1 << 30, 1)]


def attn_nsplit(keys: int) -> int:
    """Split factor of the talker decode attention for rows of at most `keys` cached keys."""
    for lim, ns in ATTN_SPLIT:
        if keys < lim:
            return ns
    return ATTN_SPLIT[-1][1]


def _lru_get(d: OrderedDict, key):
    v = d.get(key)
    if v is not None:
        d.move_to_end(key)
    return v


def _lru_put(d: OrderedDict, key, v):
    """Insert, evicting the least recently used prompt lengths beyond PREFILL_CACHE (their buffers and any graph
    captured over them go together: nothing else references them)."""
    d[key] = v
    while len(d) > PREFILL_CACHE:
        d.popitem(last=False)


def _scratch(R, st: _Stack, dev, attn_oproj=False):
    """Per-forward activations.  The attention output and the SwiGLU output only feed the next GEMM's MFMA,
    which rounds its A operand to the weight dtype anyway: in bf16 mode they are stored as bf16 (same RNE
    rounding, half the bytes the o_proj / down GEMVs read)."""
    f = lambda *s: torch.empty(*s, dtype=torch.float32, device=dev)  # noqa: E731
    a = lambda *s: torch.empty(*s, dtype=st.wdt, device=dev)  # noqa: E731
    sc = {"qkv": f(R, st.qkv_w), "q": f(R, st.Hq * st.D), "att": a(R, st.Hq * st.D), "h": a(R, st.I)}
    sc["attn_oproj"] = attn_oproj and ATTN_OPROJ and _attn_oproj_ok(st)
    if sc["attn_oproj"] and AO_HS:  # hand-off granules + sequence counters of the head-split form (zeroed once)
        sc["ao_ws"] = torch.zeros(K.attn_oproj_ws_bytes(st.H, st.Hkv), dtype=torch.uint8, device=dev)
    return sc


HANDOFF_ERROR = ("an in-launch hand-off timed out (qt_decode_attn_oproj head-split / qt_cp_step / qt_talker_tail; "
                 "blocks not co-resident?); outputs of this request are invalid (qwen_tts.talker.AO_HS / CP_ENGINE / "
                 "TALKER_TAIL = False before the model is built select the forms without hand-offs)")


class HandoffError(RuntimeError):
    """A hand-off give-up during continuous batching (serve()): the session's flag word is sticky and session-wide, so
    every request decoding when it was set is suspect.  The session stops cleanly: `failed` lists the request indices
    that were in flight (their results are not handed out), `not_started` those still queued; requests yielded
    before are unaffected (their frames were checked clear)."""

    def __init__(self, failed, not_started):
        super().__init__(HANDOFF_ERROR + f" [serve(): in-flight requests {sorted(failed)} failed, "
                                         f"{len(not_started)} queued requests not started]")
        self.failed, self.not_started = sorted(failed), list(not_started)


def _flag_words(s):
    """The sticky hand-off error words of a session's in-launch hand-off kernels (head-split attention + o_proj, the
    code-predictor step engine, the talker tail engine), int32 device views."""
    out = []
    for ws in (s.cp.sc.get("ao_ws"), s.cp.ce_ws, s.sc_t.get("tt_ws")):
        if ws is not None:
            out.append(ws[:4].view(torch.int32))
    return out


def _flag_word(s):
    """All of the session's error words as one device int32 (their OR), or None when it runs no hand-off kernel."""
    fs = _flag_words(s)
    if not fs:
        return None
    if len(fs) == 1:
        return fs[0]
    return torch.stack(fs).amax(0)


def _clear_flags(s):
    for f in _flag_words(s):
        f.zero_()


def check_handoffs(sessions):
    """Raise if an in-launch hand-off of these sessions gave up waiting (the sticky flag in a workspace): its output
    rows would hold stale partial sums.  The flags are cleared first, so a pooled session serves its next request
    normally.  Reads device words (host sync)."""
    bad = False
    for s in sessions:
        f = _flag_word(s)
        if f is not None and int(f.item()) != 0:
            _clear_flags(s)
            bad = True
    if bad:
        raise RuntimeError(HANDOFF_ERROR)


class HandoffWatch:
    """The sessions' hand-off flags copied to pinned host memory behind an event, without a host sync: armed after
    frames are queued, read once the event has completed (e.g. after the caller synchronised on a chunk's output).
    check() raises (and clears the device flag) when a flag was set."""

    def __init__(self, sessions):
        self.items = []
        for s in sessions:
            f = _flag_word(s)
            if f is None:
                continue
            h = torch.empty(1, dtype=torch.int32, pin_memory=True)
            h.copy_(f, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            self.items.append((s, h, ev))

    def check(self, block: bool = True) -> bool:
        """True once every copy has landed and no flag was set; False when not landed yet (block=False)."""
        bad = False
        for s, h, ev in self.items:
            if not block and not ev.query():
                return False
            ev.synchronize()
            if int(h[0]) != 0:
                _clear_flags(s)
                bad = True
        if bad:
            raise RuntimeError(HANDOFF_ERROR)
        return True


def _attn_oproj_ok(st: _Stack) -> bool:
    kt = 32 if st.wdt == torch.bfloat16 else 16
    ks = (st.Hq // st.Hkv) * st.D
    return (st.D in (16, 64, 128) and st.Hq // st.Hkv in (1, 2, 4) and st.Hkv <= 8 and ks % kt == 0
            and ks // kt <= 16)


class CPLane:
    """Buffers of a session's code predictor (rows [b0, b1) = the whole batch): the chain of the 15 sequential CP
    steps of one frame.  (Round 2 also ran half-batch lanes on forked streams inside the frame graph; graph branches
    do not overlap on this stack and the split measured slower -- 156.5 vs 167.0 audio-s/s -- so it was removed.)"""

    def __init__(self, s: "Session", eng: "TalkerEngine", b0: int, b1: int, ws):
        c, dev = eng.cp, eng.dev
        self.b0, self.b1, self.nb = b0, b1, b1 - b0
        nb = self.nb
        i32 = lambda *z: torch.zeros(*z, dtype=torch.int32, device=dev)  # noqa: E731
        # prefill rows (2r, 2r + 1) = (past_hidden, cb0 embedding); decode rows 0..nb-1 of the same slice
        self.x = s.cp_x[2 * b0:2 * b1]
        self.x16 = None if s.cp_x16 is None else s.cp_x16[2 * b0:2 * b1]
        self.kv = ([k[b0:b1] for k in s.cp_kv[0]], [v[b0:b1] for v in s.cp_kv[1]])
        self.sc = _scratch(2 * nb, c, dev, attn_oproj=nb <= ATTN_OPROJ_MAX)
        self.ws = ws
        # the step engine's hand-off granules + launch counter (zeroed once, kept across launches)
        self.ce_ws = (torch.zeros(K.cp_step_ws_bytes(), dtype=torch.uint8, device=dev)
                      if eng.cp_engine and nb <= 8 else None)
        self.logits = torch.zeros(nb, eng.Vc, dtype=torch.float32, device=dev)
        self.tok = s.cp_tok[b0:b1]
        self.codes = s.codes[b0:b1]
        rb2 = torch.arange(2 * nb, device=dev, dtype=torch.int32) // 2
        p2 = torch.arange(2 * nb, device=dev, dtype=torch.int32) % 2
        self.meta0 = {"rope_pos": p2, "kv_pos": p2.clone(), "row_len": p2 + 1, "row_start": i32(2 * nb),
                      "row_batch": rb2, "small_T": 2}
        rb = torch.arange(nb, dtype=torch.int32, device=dev)
        self.meta = []
        for g in range(1, s.G - 1):
            pos = torch.full((nb,), g + 1, dtype=torch.int32, device=dev)
            self.meta.append({"rope_pos": pos, "kv_pos": pos.clone(), "row_len": pos + 1, "row_start": i32(nb),
                              "row_batch": rb, "const_pos": g + 1})


@dataclass
class GenParams:
    max_new_tokens: int = 4096
    do_sample: bool = True
    top_k: int = 50
    top_p: float = 1.0
    temperature: float = 0.9
    subtalker_dosample: bool = True
    subtalker_top_k: int = 50
    subtalker_top_p: float = 1.0
    subtalker_temperature: float = 0.9
    eos_token_id: Optional[int] = None
    repetition_penalty: float = 1.05
    ignore_eos: bool = False
    # Philox key of this request's draws.  None (default): a fresh one per generate() call drawn from torch's
    # default CPU generator, so repeated calls differ like the reference's torch.multinomial draws and
    # torch.manual_seed makes them reproducible.  It lives in a device word read by the samplers, so it is not
    # part of the session key: a new seed replays the same captured graph.
    seed: Optional[int] = None

    def key(self):
        return (self.do_sample, self.top_k, self.top_p, self.temperature, self.subtalker_dosample,
                self.subtalker_top_k, self.subtalker_top_p, self.subtalker_temperature, self.eos_token_id,
                self.repetition_penalty, self.ignore_eos)

    def resolve_seed(self) -> int:
        if self.seed is not None:
            return int(self.seed) & (2 ** 63 - 1)
        return int(torch.randint(0, 2 ** 63 - 1, (1,)).item())


class Session:
    """Device buffers + captured frame graph for one (batch, capacity, params) shape."""

    def __init__(self, eng: "TalkerEngine", B: int, P_cap: int, max_frames: int, gp: GenParams, teacher=False):
        dev, t, c = eng.dev, eng.talker, eng.cp
        self.B, self.P_cap, self.max_frames, self.gp = B, P_cap, max_frames, gp
        self.Lmax = P_cap + max_frames + 2
        i32 = lambda *s: torch.zeros(*s, dtype=torch.int32, device=dev)  # noqa: E731
        kvd = eng.kv_dtype
        self.kv = ([torch.zeros(B, t.Hkv, self.Lmax, t.D, dtype=kvd, device=dev) for _ in range(t.n_layers)],
                   [torch.zeros(B, t.Hkv, self.Lmax, t.D, dtype=kvd, device=dev) for _ in range(t.n_layers)])
        self.G = eng.G
        self.cp_L = self.G + 1
        self.cp_kv = ([torch.zeros(B, c.Hkv, self.cp_L, c.D, dtype=kvd, device=dev) for _ in range(c.n_layers)],
                      [torch.zeros(B, c.Hkv, self.cp_L, c.D, dtype=kvd, device=dev) for _ in range(c.n_layers)])
        # per-row counters, field-major [5][B]: frame index (step), n_generated, rope_pos, kv_pos, kv_len -- every row
        # its own request clock, so a batch slot can be refilled with a new request mid-decode (serve()); a row
        # advances until its frame index reaches max_frames (qt_advance_rows)
        self.ctr = i32(5 * B)
        self.step, self.n_gen = self.ctr[0:B], self.ctr[B:2 * B]
        self.meta = {"rope_pos": self.ctr[2 * B:3 * B], "kv_pos": self.ctr[3 * B:4 * B],
                     "row_len": self.ctr[4 * B:5 * B], "row_start": i32(B),
                     "row_batch": torch.arange(B, dtype=torch.int32, device=dev)}
        self.prow = torch.arange(B, dtype=torch.int32, device=dev)  # Philox stream id of each row's request
        f32 = lambda *s: torch.zeros(*s, dtype=torch.float32, device=dev)  # noqa: E731
        self.x = f32(B, t.H)
        # bf16 shadows of the decode residual streams (bf16 mode): A operands of the RMS-normalised GEMVs
        use16 = eng.wdt == torch.bfloat16 and X16
        bf = lambda *s: torch.zeros(*s, dtype=torch.bfloat16, device=dev) if use16 else None  # noqa: E731
        self.x16 = bf(B, t.H)
        self.cp_x16 = bf(2 * B, c.H)
        self.past_hidden = f32(B, t.H)
        self.logits = f32(B, eng.V)
        self.cp_x = f32(2 * B, c.H)
        self.sc_t = _scratch(B, t, dev)
        # split-KV records + arrival counters of the talker decode attention (zeroed; every launch re-arms them)
        self.sc_t["attn_ws"] = torch.zeros(K.decode_attn_ws_bytes(B, t.Hq, t.Hkv, t.D, 8), dtype=torch.uint8,
                                           device=dev)
        if eng.talker_tail and B <= 8:  # the talker decode-layer tail engine's hand-off workspace (zeroed once)
            self.sc_t["tt_ws"] = torch.zeros(K.talker_tail_ws_bytes(), dtype=torch.uint8, device=dev)
        self.codes = i32(B, max_frames + 2, self.G)
        # teacher forcing (parity diagnostics): every sampler continues with force[] and records its choice in pick[]
        self.force = i32(B, max_frames + 2, self.G) if teacher else None
        self.pick = i32(B, max_frames + 2, self.G) if teacher else None
        self.hiddens = f32(B, max_frames + 2, t.H)  # + the frame a capped row re-runs (serve())
        self.tok0 = i32(B)
        self.cp_tok = i32(B)
        self.seen = torch.zeros(B, eng.V, dtype=torch.uint8, device=dev)
        self.finished = torch.zeros(B, dtype=torch.uint8, device=dev)
        self.trailing = f32(B, max_frames + 1, t.H)
        self.pad_embed = f32(t.H)
        self.ws = K.new_workspace(dev)  # split-K scratch private to this session's stream
        self.seed = torch.zeros(1, dtype=torch.int64, device=dev)  # Philox key, read by the captured samplers
        self.graph = None   # the frame graph of the current split factor (graphs[nsplit])
        self.graphs = {}    # talker attention split factor -> captured frame graph
        # prompt length P -> static prefill buffers (+ captured graph once P repeats); LRU, PREFILL_CACHE lengths
        self.prefill = OrderedDict()
        self.slot_prefill = OrderedDict()  # P -> static single-request prefill buffers (serve() refills); LRU
        self.busy = False  # held by a live decode_iter (a suspended stream() generator included)
        self.watch = None  # HandoffWatch armed at the last yield of decode_iter
        self.cp = CPLane(self, eng, 0, B, self.ws)


class TalkerEngine:
    def __init__(self, cfg: dict, weights: Dict[str, torch.Tensor], dtype: str = "bf16", device="cuda"):
        _hip.lib()
        self.cfg = cfg
        self.tc = tc = cfg["talker_config"]
        self.cc = cc = tc["code_predictor_config"]
        self.dev = torch.device(device)
        self.wdt = torch.bfloat16 if dtype == "bf16" else torch.float32
        self.kv_dtype = self.wdt
        self.G = tc["num_code_groups"]
        self.V, self.Vc = tc["vocab_size"], cc["vocab_size"]
        W, dev, wdt = weights, self.dev, self.wdt
        # RoPE positions for prompt + max_new_tokens (4096) without regrowing in the common case
        self.talker = _Stack(W, "talker.model", tc, wdt, dev, 8192)
        self.cp = _Stack(W, "talker.code_predictor.model", cc, wdt, dev, self.G + 2)
        self.codec_head = K.tile_linear(_w(W, "talker.codec_head.weight", dev), wdt)
        self.emb0 = _w(W, "talker.model.codec_embedding.weight", dev).to(wdt).contiguous()
        self.text_emb = _w(W, "talker.model.text_embedding.weight", dev).to(wdt).contiguous()
        self.fc1 = K.tile_linear(_w(W, "talker.text_projection.linear_fc1.weight", dev), wdt,
                                 _w(W, "talker.text_projection.linear_fc1.bias", dev))
        self.fc2 = K.tile_linear(_w(W, "talker.text_projection.linear_fc2.weight", dev), wdt,
                                 _w(W, "talker.text_projection.linear_fc2.bias", dev))
        self.ecp = torch.stack([_w(W, f"talker.code_predictor.model.codec_embedding.{g}.weight", dev).to(wdt)
                                for g in range(self.G - 1)]).contiguous()
        self.lm_heads = [K.tile_linear(_w(W, f"talker.code_predictor.lm_head.{g}.weight", dev), wdt, gamma=self.cp.norm)
                         for g in range(self.G - 1)]  # CP final norm folded in (M:1142, 1299)
        s2m = "talker.code_predictor.small_to_mtp_projection.weight"
        self.s2m = K.tile_linear(_w(W, s2m, dev), wdt, _w(W, s2m.replace("weight", "bias"), dev)) if s2m in W else None
        # next-step code-predictor inputs as tables (fp32 [vocab][Hc]): codec embedding rows already passed
        # through small_to_mtp (when present), gathered by the samplers instead of a per-step GEMV
        Hc = cc["hidden_size"]
        self.cp_in_tabs = [self._proj_table(self.ecp[g], Hc) for g in range(self.G - 2)]
        self.cp_in_tab0 = self._proj_table(self.emb0, Hc)
        # bf16 mode: the code predictor's layer-0 q/k/v projection of every decode-step input row, precomputed per
        # table ([V][qkv_w] fp32, from the bf16-rounded rows as the x16 shadow feeds the decode GEMV): the sampler that
        # picks a step's token also gathers its q/k/v row, so decode steps skip the layer-0 QKV GEMV (14 launches/frame)
        self.cp_qkv_tabs = None
        if self.wdt == torch.bfloat16 and QKV0_TAB:
            L0, c = self.cp.layers[0], self.cp
            self.cp_qkv_tabs = []
            for tab in self.cp_in_tabs:
                t16 = tab.to(torch.bfloat16)
                out = torch.empty(tab.shape[0], c.qkv_w, dtype=torch.float32, device=dev)
                K.gemm(t16, L0.qkv, out, tab.shape[0], Hc, c.qkv_w, rms=True, eps=c.eps)
                self.cp_qkv_tabs.append(out)
        # the code-predictor step engine (qt_cp_step): bf16, layer-0 q/k/v tables, the shapes it is built for, and a
        # device that keeps its 256 workgroups resident
        c = self.cp
        self.cp_engine = (CP_ENGINE and self.cp_qkv_tabs is not None and
                          K.cp_step_supported(c.H, c.I, c.Hq, c.Hkv, c.D, c.n_layers, self.Vc))
        # the talker decode-layer tail engine (qt_talker_tail): bf16, its shapes, all 256 workgroups resident
        t = self.talker
        self.talker_tail = (TALKER_TAIL and self.wdt == torch.bfloat16 and
                            K.talker_tail_supported(t.H, t.I, t.Hq, t.D, t.qkv_w))
        self._sessions: Dict[tuple, List[Session]] = {}
        self._fence = None  # (event, stream) of the last frame issued (_fence_in / _fence_out)
        torch.cuda.synchronize()

    def _proj_table(self, emb, Hc):
        """small_to_mtp(embedding table) (M:1299 applied row-wise) or the table itself, fp32 [V][Hc]."""
        V = emb.shape[0]
        if self.s2m is None:
            return emb.float().contiguous()
        out = torch.empty(V, Hc, dtype=torch.float32, device=self.dev)
        K.gemm(emb, self.s2m, out, V, emb.shape[1], Hc, a_dtype=emb.dtype)
        return out

    # ---------------------------------------------------------------- G1: prompt embeddings
    def text_proj(self, ids: torch.Tensor) -> torch.Tensor:
        """text_projection(text_embedding(ids)) (M:808-816): gather -> fc1(+b, SiLU) -> fc2(+b); fp32 [n, H]."""
        ids = _to_dev_i32(ids, self.dev)
        n = ids.numel()
        thd = self.text_emb.shape[1]
        if n > 16 and self.text_emb.dtype == torch.bfloat16 and self.fc1.dtype == torch.bfloat16:
            # a batch's prompt text (~1.7k ids at B = 8 x 200 tokens): gather the rows, then the bf16-A prefill GEMMs
            # (the gathered-A path is the generic gemm_wt: 240 us for fc1 at B = 8); fc1's output is stored in bf16,
            # the value fc2's MFMA reads either way
            a16 = self.text_emb.index_select(0, ids)  # bf16 rows, as stored
            h16 = torch.empty(n, self.fc1.N, dtype=torch.bfloat16, device=self.dev)
            K.gemm(a16, self.fc1, h16, n, thd, self.fc1.N, act=_hip.ACT_SILU)
            out = torch.empty(n, self.fc2.N, dtype=torch.float32, device=self.dev)
            K.gemm(h16, self.fc2, out, n, self.fc1.N, self.fc2.N)
            return out
        h = torch.empty(n, self.fc1.N, dtype=torch.float32, device=self.dev)
        K.gemm(self.text_emb, self.fc1, h, n, thd, self.fc1.N, a_dtype=self.text_emb.dtype, a_index=ids,
               act=_hip.ACT_SILU)
        out = torch.empty(n, self.fc2.N, dtype=torch.float32, device=self.dev)
        K.gemm(h, self.fc2, out, n, self.fc1.N, self.fc2.N)
        return out

    def codec_embed(self, ids) -> torch.Tensor:
        ids = _to_dev_i32(ids, self.dev)
        H = self.talker.H
        out = torch.empty(ids.numel(), H, dtype=torch.float32, device=self.dev)
        K.gather_rows(self.emb0, ids, ids.numel(), H, out, H)
        return out

    def cp_embed(self, g, ids) -> torch.Tensor:
        ids = _to_dev_i32(ids, self.dev)
        H = self.talker.H
        out = torch.empty(ids.numel(), H, dtype=torch.float32, device=self.dev)
        K.gather_rows(self.ecp[g], ids, ids.numel(), H, out, H)
        return out

    # ---------------------------------------------------------------- sessions / graph
    def session(self, B, P, max_frames, gp: GenParams, teacher: bool = False) -> Session:
        """A free session of this shape, marked busy (release() hands it back).  A session held by a live request
        (e.g. a suspended stream() generator) is never shared: a concurrent request of the same shape gets a
        session of its own (own KV cache, counters and captured graph)."""
        P_cap = max(64, (P + 63) // 64 * 64)
        key = (B, max_frames, gp.key(), teacher)
        pool = self._sessions.setdefault(key, [])
        for s in pool:
            if not s.busy and s.P_cap >= P:
                s.busy = True
                return s
        # HBM: drop idle sessions of other (max_frames, params) families and idle ones too small for P
        for k in list(self._sessions):
            if k[1:3] != key[1:3] or k == key:
                self._sessions[k] = [s for s in self._sessions[k] if s.busy]
        idle = [s for ss in self._sessions.values() for s in ss if not s.busy]
        if len(idle) >= 8:
            for k in list(self._sessions):
                self._sessions[k] = [s for s in self._sessions[k] if s.busy]
        for k in [k for k, v in self._sessions.items() if not v and k != key]:
            del self._sessions[k]
        s = Session(self, B, P_cap, max_frames, gp, teacher=teacher)
        self.talker.ensure_rope(s.Lmax + 4, self.dev)
        self._sessions.setdefault(key, []).append(s)
        s.busy = True
        return s

    @staticmethod
    def release(sessions):
        for s in sessions:
            s.busy = False

    def all_sessions(self) -> List[Session]:
        return [s for ss in self._sessions.values() for s in ss]

    def _eos(self, gp):
        return gp.eos_token_id if gp.eos_token_id is not None else self.tc["codec_eos_token_id"]

    def _sample_talker(self, s: Session, logits, codes_step_off, substep, b0=0, b1=None):
        """Talker token choice for rows [b0, b1) of the session (default all)."""
        gp = s.gp
        eos = self._eos(gp)
        b1 = s.B if b1 is None else b1
        Hc = self.cp.H
        K.sample(logits[b0:b1], b1 - b0, self.V, self.V, s.tok0[b0:b1], seen=s.seen[b0:b1],
                 rep_penalty=gp.repetition_penalty, n_generated=s.n_gen[b0:b1], min_new_tokens=MIN_NEW_TOKENS, eos_id=eos,
                 suppress=(self.V - 1024, self.V, self.tc["codec_eos_token_id"]), ignore_eos=gp.ignore_eos,
                 finished=s.finished[b0:b1], do_sample=gp.do_sample, top_k=gp.top_k, top_p=gp.top_p,
                 temperature=gp.temperature, seed_ptr=s.seed, step=s.step[b0:b1], substep=substep,
                 codes=s.codes[b0:b1], codes_ld=s.codes.shape[1] * self.G, codes_w=self.G, codes_col=0,
                 codes_step_off=codes_step_off, ctr_stride=1, philox_row=s.prow[b0:b1],
                 emb=(self.cp_in_tab0, s.cp_x.view(-1)[(2 * b0 + 1) * Hc:], 2 * Hc),
                 emb16=None if s.cp_x16 is None else (s.cp_x16.view(-1)[(2 * b0 + 1) * Hc:], 2 * Hc),
                 force=None if s.force is None else s.force[b0:b1], pick=None if s.pick is None else s.pick[b0:b1])

    def _frame(self, s: Session, part: str = "all"):
        """One decode step (M:1669-1744): CP 15 tokens -> 16-codebook embed sum -> talker -> next cb0.  part = "cp"
        issues only the code predictor (after it the frame's 16 codes are complete), "talk" only the rest."""
        B, t = s.B, self.talker
        codes_ld = s.codes.shape[1] * self.G
        if part != "talk":
            self._cp_lane(s, s.cp)
        if part == "cp":
            return
        # --- talker decode input and forward
        K.frame_embed(self.emb0, self.ecp, self.G, t.H, s.codes, codes_ld, s.step, s.trailing,
                      s.trailing.shape[1], s.pad_embed, s.x, B, x16=s.x16, step_stride=1)
        t.forward(s.x, B, s.meta, s.kv, s.sc_t, s.Lmax, s.Lmax, decode=True, x16=s.x16)
        # next frame's past_hidden, also recorded as that frame's hidden state (hiddens[:, step + 1])
        K.rmsnorm(s.x, t.norm, t.eps, s.past_hidden, B, t.H, rec=s.hiddens, step=s.step, step_off=1, step_stride=1)
        K.gemm(s.past_hidden, self.codec_head, s.logits, B, t.H, self.V)
        self._sample_talker(s, s.logits, 1, 0)
        K.advance_rows(s.ctr, B, 5, s.max_frames)

    def _cp_lane(self, s: Session, ln: CPLane):
        """Code predictor for rows [b0, b1): 2-token prefill + 14 decode steps (M:1671-1680)."""
        t, c = self.talker, self.cp
        Hc, nb = c.H, ln.nb
        # --- prefill: rows (2r, 2r+1) = (past_hidden[r], codec_embedding(tok0[r])); the odd rows were written by
        # the talker sampler that chose tok0 (projected embedding table)
        if self.s2m is not None:
            K.gemm(s.past_hidden[ln.b0:ln.b1], self.s2m, ln.x, nb, t.H, 2 * Hc, out2=ln.x16)
        else:
            ln.x.view(nb, 2, Hc)[:, 0].copy_(s.past_hidden[ln.b0:ln.b1])
            if ln.x16 is not None:
                ln.x16.view(nb, 2, Hc)[:, 0].copy_(s.past_hidden[ln.b0:ln.b1])
        fuse = ln.ce_ws is not None and CP_FUSE_SAMPLE and self.Vc <= 2048
        pending = None  # the token choice the next step's launch makes first (fused)
        if ln.ce_ws is not None and CP_PREFILL:  # every layer + lm_head[0] for both positions in one launch
            K.cp_prefill(c.layers, self.lm_heads[0], ln.x, nb, ln.kv[0], ln.kv[1], s.cp_L, c.cos, c.sin, c.eps,
                         ln.logits, ln.ce_ws)
            if fuse:
                pending = self._cp_sample(s, ln, 0, launch=False)
            else:
                self._cp_sample(s, ln, 0)
        else:
            p16 = ln.x16 if 2 * nb <= 96 else None  # forward() keeps the shadow for decode / skinny-GEMV row counts
            c.forward(ln.x, 2 * nb, ln.meta0, ln.kv, ln.sc, s.cp_L, s.cp_L, x16=p16)
            self._cp_head(s, ln, ln.x.view(-1)[Hc:], 2 * Hc, 0, None if p16 is None else p16.view(-1)[Hc:])
        for g in range(1, self.G - 1):
            x = ln.x[:nb]  # written by the previous step's sampler (embedding of the token it chose)
            x16 = None if ln.x16 is None else ln.x16[:nb]
            if ln.ce_ws is not None:  # the whole step (5 layers + lm_head[g]) in one persistent launch
                K.cp_step(c.layers, self.lm_heads[g], x, ln.sc["qkv"][:nb], nb, ln.kv[0], ln.kv[1], s.cp_L, g + 1,
                          c.cos, c.sin, c.eps, ln.logits, ln.ce_ws, sample=pending)
                if fuse and g < self.G - 2:
                    pending = self._cp_sample(s, ln, g, launch=False)
                else:
                    pending = None
                    self._cp_sample(s, ln, g)
                continue
            c.forward(x, nb, ln.meta[g - 1], ln.kv, ln.sc, s.cp_L, s.cp_L, decode=True, x16=x16,
                      qkv0=self.cp_qkv_tabs is not None)
            self._cp_head(s, ln, x, Hc, g, x16)

    def _cp_head(self, s: Session, ln: CPLane, h, ldh, g, h16=None):
        c = self.cp
        K.gemm(h if h16 is None else h16, self.lm_heads[g], ln.logits, ln.nb, ldh, self.Vc, rms=True, eps=c.eps)
        self._cp_sample(s, ln, g)

    def _cp_sample(self, s: Session, ln: CPLane, g, launch=True):
        c, gp = self.cp, s.gp
        return K.sample(ln.logits, ln.nb, self.Vc, self.Vc, ln.tok, do_sample=gp.subtalker_dosample,
                 top_k=gp.subtalker_top_k, top_p=gp.subtalker_top_p, temperature=gp.subtalker_temperature,
                 seed_ptr=s.seed, step=s.step[ln.b0:ln.b1], substep=1 + g, codes=ln.codes,
                 codes_ld=s.codes.shape[1] * self.G, codes_w=self.G, codes_col=1 + g, codes_step_off=0, ctr_stride=1,
                 philox_row=s.prow[ln.b0:ln.b1],
                 emb=(self.cp_in_tabs[g], ln.x, c.H) if g < self.G - 2 else None,
                 emb16=(ln.x16, c.H) if ln.x16 is not None and g < self.G - 2 else None,
                 emb2=(self.cp_qkv_tabs[g], ln.sc["qkv"], c.qkv_w) if self.cp_qkv_tabs is not None and g < self.G - 2
                 else None,
                 force=None if s.force is None else s.force[ln.b0:ln.b1],
                 pick=None if s.pick is None else s.pick[ln.b0:ln.b1], launch=launch)

    # ---------------------------------------------------------------- G2/G3: prefill + decode loop
    def generate_from_embeds(self, embeds: torch.Tensor, mask: torch.Tensor, trailing: torch.Tensor,
                             tts_pad: torch.Tensor, gp: GenParams, use_graph: bool = True, on_frames=None,
                             philox_ids=None):
        """embeds fp32 [B,P,H] left-padded, mask [B,P] -> (codes list [F_i,16] int64 cpu, hidden list).

        philox_ids: optional per-row Philox stream ids (default the row index) -- a data-parallel shard passes its
        requests' global indices, so every request draws the same stream whichever rank and row decode it."""
        it = self.decode_iter(embeds, mask, trailing, tts_pad, gp, use_graph=use_graph, on_frames=on_frames,
                              philox_ids=philox_ids)
        out = None
        for sessions, frames, final in it:
            if final:  # collected while the sessions are still held by this request
                out = self.collect(sessions, frames)
        return out

    def teacher_forced(self, embeds, mask, trailing, tts_pad, gp: GenParams, ref_codes, use_graph: bool = True):
        """Teacher-forced decode (parity diagnostics): every token choice -- the talker's cb0 and the code
        predictor's 15 -- is made by this path's processors and argmax as in generate(), recorded, and then replaced by
        the reference's token, so each step sees exactly the reference's history.  ref_codes: per row [F_b, 16].
        Returns (picks [B, F, 16] int64 cpu in the codes' layout, hidden [B, F, H] cpu), F = max F_b; entries past a
        row's F_b are unspecified."""
        import dataclasses
        B, P, H = embeds.shape
        F = max(int(c.shape[0]) for c in ref_codes)
        gp = dataclasses.replace(gp, max_new_tokens=F + 1)
        s = self.session(B, P, max(F, 1), gp, teacher=True)
        try:
            s.force.zero_()
            for b, c in enumerate(ref_codes):
                s.force[b, :c.shape[0]] = torch.as_tensor(c).to(self.dev, torch.int32)
            with K.use_workspace(s.ws):
                self._prefill(s, embeds, mask, trailing, tts_pad, gp.resolve_seed())
            s.hiddens[:, 0].copy_(s.past_hidden)
            for f in range(F):
                self._run_frame(s, P + f + 1, use_graph)
            check_handoffs([s])
            return s.pick[:, :F].long().cpu(), s.hiddens[:, :F].cpu()
        finally:
            self.release([s])

    def decode_iter(self, embeds, mask, trailing, tts_pad, gp: GenParams, use_graph: bool = True, on_frames=None,
                    every: int = 0, first: int = 0, grow: bool = False, philox_ids=None, early_first: bool = False):
        """Prefill + frame loop as a generator: yields (sessions, frames_done, final) after `first` frames, then
        every `every` frames (0: only at the end; grow=True: intervals double from first - 1 up to `every`), and once
        at the end with final=True.  `sessions` is a one-element list (the batch's session); codes[:, :frames_done]
        are final when yielded (device), and codes[:, frames_done, 0] already holds the next frame's cb0 (EOS of rows
        that just finished).  early_first (with first == 1): the first yield comes as soon as frame 0's codes are
        complete -- after its code predictor, before the talker step that starts frame 1 (which is queued after the
        caller's work, e.g. the first codec window); at that yield codes[:, 1, 0] is not written yet (EOS cannot occur
        there anyway: it is masked below min_new_tokens)."""
        B, P, H = embeds.shape
        max_frames = max(gp.max_new_tokens - 1, 0)
        seed = gp.resolve_seed()
        main = torch.cuda.current_stream(self.dev)
        sessions = []
        try:
            s = self.session(B, P, max(max_frames, 1), gp)
            sessions.append(s)
            with K.use_workspace(s.ws):
                self._prefill(s, embeds, mask, trailing, tts_pad, seed, philox_ids)
            yield from self._frames(sessions, [main], max_frames, use_graph, on_frames, every, first, grow, early_first)
        finally:
            self.release(sessions)

    def _frames(self, sessions, streams, max_frames, use_graph, on_frames, every, first, grow=False, early_first=False):
        main = torch.cuda.current_stream(self.dev)
        frames = 0
        check_every = 8
        next_yield = first or every
        interval = max(first - 1, 1)
        for s, st in zip(sessions, streams):
            with torch.cuda.stream(st):
                s.hiddens[:, 0].copy_(s.past_hidden)  # later frames are recorded inside the frame graph
        # EOS polling without a host sync: every `check_every` frames the all-finished flag is copied to pinned
        # memory behind an event; the copy from the previous window is read once its event has completed
        pending = []
        watch = None  # hand-off flags as of the previous yield (checked before the next chunk is handed out)
        while frames < max_frames:
            early = early_first and frames == 0 and next_yield == 1 and max_frames > 1
            for s, st in zip(sessions, streams):
                with torch.cuda.stream(st):  # every row holds <= P + frames + 1 keys
                    self._run_frame(s, s.P + frames + 1, use_graph, "cp" if early else "all")
            frames += 1
            if on_frames is not None:
                on_frames(sessions[0], frames)
            if next_yield and frames == next_yield and frames < max_frames:
                for st in streams:
                    main.wait_stream(st)
                if watch is not None:  # the caller consumed the previous chunk: those frames are done
                    watch.check()
                with torch.cuda.stream(main):
                    watch = HandoffWatch(sessions)
                for s in sessions:  # a caller that synchronised on these frames checks it before using them
                    s.watch = watch
                yield sessions, frames, False
                interval = min(every, 2 * interval) if grow else every
                next_yield = frames + interval if every else 0
            if early:  # the rest of frame 0 (talker step -> cb0 of frame 1), behind the caller's work
                for s, st in zip(sessions, streams):
                    with torch.cuda.stream(st):
                        self._run_frame(s, s.P + 1, use_graph, "talk")
            if frames % check_every == 0 and frames < max_frames:
                flags = []
                for s, st in zip(sessions, streams):
                    with torch.cuda.stream(st):
                        f = torch.empty(1, dtype=torch.bool, pin_memory=True)
                        f.copy_(s.finished.all().reshape(1), non_blocking=True)
                        ev = torch.cuda.Event()
                        ev.record(st)
                        flags.append((f, ev))
                pending.append(flags)
                done = False
                while pending and all(ev.query() for _, ev in pending[0]):
                    if all(bool(f.item()) for f, _ in pending.pop(0)):
                        done = True
                if done:
                    break
        for st in streams:
            main.wait_stream(st)
        check_handoffs(sessions)
        yield sessions, frames, True

    def collect(self, sessions, frames):
        """Per-row codes (EOS-truncated, M:2280-2292) and last hidden states, host tensors."""
        eos = self.tc["codec_eos_token_id"]
        out_c, out_h = [], []
        for s in sessions:
            codes = s.codes[:, :frames].long().cpu()
            hid = s.hiddens[:, :frames].cpu()
            for b in range(s.B):
                c0 = codes[b, :, 0]
                stop = (c0 == eos).nonzero()
                L = int(stop[0]) if stop.numel() else frames
                out_c.append(codes[b, :L])
                out_h.append(hid[b, :L])
        return out_c, out_h

    # ---------------------------------------------------------------- continuous batching
    def serve(self, requests, tts_pad, gp: GenParams, slots: int = 8, use_graph: bool = True, poll: int = 4,
              philox_ids=None):
        """Continuous batching: decode `requests` through `slots` batch rows of one session, refilling a row with
        the next queued request as soon as its request ends (EOS, or max_new_tokens - 1 frames) instead of padding
        it with EOS until the whole batch ends as the reference's batched generate() does (M:2272-2292).

        requests: list of (embeds fp32 [P_i, H], trailing fp32 [T_i, H][, frames_i]) -- one unpadded prompt each (a
        row of build_prompts() with its left padding removed); the optional frames_i caps that request below
        max_new_tokens - 1 frames (it is retired at the first poll past it, so its row may run up to `poll` frames
        longer).  Yields (i, codes [F_i, 16] int64 cpu, hidden [F_i, H] cpu)
        as requests finish (completion order).  Request i draws Philox stream i of the call's seed, i.e. the
        stream row i of a one-shot batched generate() of the same list draws, whichever slot decodes it.  Per request
        the result equals the one-shot batch's up to GEMM summation order: a refill prefills P rows while the batch
        prefills B x P, and at production sizes the two row counts can take different GEMM kernels (skinny GEMV /
        split-K vs gemm_pf_k), so in bf16 a near-tie may resolve differently (fp32: identical in the tests).

        The frame graph is the session's ordinary captured frame (per-row step / position counters); a refill is
        a single-request prefill into the slot's K/V rows between two graph replays.  The host learns which rows
        ended from pinned copies of the device flags every `poll` frames (no host sync on the decode stream).
        philox_ids: optional Philox stream id per request (default its index i)."""
        n = len(requests)
        pids = list(range(n)) if philox_ids is None else [int(x) for x in philox_ids]
        if n == 0:
            return
        B = max(1, min(slots, n))
        ahead = 1
        max_frames = max(gp.max_new_tokens - 1, 1)
        P = max(int(r[0].shape[0]) for r in requests)
        cap_i = [min(max_frames, int(r[2])) if len(r) > 2 and r[2] is not None else max_frames for r in requests]
        seed = gp.resolve_seed()
        eos = self.tc["codec_eos_token_id"]
        s = self.session(B, P, max_frames, gp)
        H, dev = self.talker.H, self.dev
        try:
            with K.use_workspace(s.ws):
                # the first B requests start together: one left-padded batched prefill (as generate() does)
                Pb = max(int(r[0].shape[0]) for r in requests[:B])
                Tb = max(int(r[1].shape[0]) for r in requests[:B])
                emb = torch.zeros(B, Pb, H, dtype=torch.float32, device=dev)
                mask = torch.zeros(B, Pb, dtype=torch.long, device=dev)
                trail = tts_pad.reshape(1, 1, H).float().to(dev).repeat(B, Tb, 1)
                for b in range(B):
                    e, tr = requests[b][0], requests[b][1]
                    emb[b, Pb - e.shape[0]:] = e
                    mask[b, Pb - e.shape[0]:] = 1
                    trail[b, :tr.shape[0]] = tr
                self._prefill(s, emb, mask, trail, tts_pad, seed, pids[:B])
                s.hiddens[:, 0].copy_(s.past_hidden)
                queue = list(range(B, n))
                slot_req = list(range(B))
                epoch = [0] * B
                start = [0] * B  # host frame count when the slot's request started
                slot_p = [Pb] * B  # prompt length (K/V rows before the first frame) of each slot's request
                polls, harvests = [], []
                frame = 0
                while any(r >= 0 for r in slot_req) or harvests:
                    if any(r >= 0 for r in slot_req):
                        keys = max(slot_p[b] + frame - start[b] + 1 for b in range(B) if slot_req[b] >= 0)
                        self._run_frame(s, min(keys, s.Lmax), use_graph)
                        frame += 1
                        if frame % poll == 0 and not gp.ignore_eos:  # (with ignore_eos only frame counts end rows)
                            st = torch.empty(2 * B, dtype=torch.int32, pin_memory=True)
                            st[:B].copy_(s.step, non_blocking=True)
                            st[B:].copy_(s.finished, non_blocking=True)
                            ev = torch.cuda.Event()
                            ev.record()
                            polls.append((st, list(epoch), ev))
                    else:  # only harvests left in flight
                        harvests[0][-1].synchronize()
                    # rows that ended (as of a completed poll, same request still in the slot): copy their codes out
                    # and refill the slot, both in stream order behind the frames already queued.  The host may run
                    # at most `ahead` polls in front of the GPU (else it would queue many frames past a row's end
                    # before seeing it, and that row's slot would idle for all of them)
                    ended = [b for b in range(B) if slot_req[b] >= 0 and frame - start[b] >= cap_i[slot_req[b]]]
                    while polls and (len(polls) > ahead or polls[0][2].query()):
                        polls[0][2].synchronize()
                        st, ep, _ = polls.pop(0)
                        ended += [b for b in range(B) if slot_req[b] >= 0 and ep[b] == epoch[b] and int(st[B + b])]
                    # a row whose request reached its frame count is known on the host without a poll (its frame
                    # index = frames replayed since it started); EOS is learned from the polls
                    for b in sorted(set(ended)):
                        hc = torch.empty(s.codes.shape[1], self.G, dtype=torch.int32, pin_memory=True)
                        hh = torch.empty(s.hiddens.shape[1], H, dtype=torch.float32, pin_memory=True)
                        hs = torch.empty(1, dtype=torch.int32, pin_memory=True)
                        hc.copy_(s.codes[b], non_blocking=True)
                        hh.copy_(s.hiddens[b], non_blocking=True)
                        hs.copy_(s.step[b:b + 1], non_blocking=True)
                        hf, fw = None, _flag_word(s)
                        if fw is not None:  # the hand-off flags as of this request's last frame
                            hf = torch.empty(1, dtype=torch.int32, pin_memory=True)
                            hf.copy_(fw, non_blocking=True)
                        ev = torch.cuda.Event()
                        ev.record()
                        harvests.append((slot_req[b], hc, hh, hs, hf, ev))
                        epoch[b] += 1
                        start[b] = frame
                        slot_req[b] = queue.pop(0) if queue else -1
                        if slot_req[b] >= 0:
                            slot_p[b] = int(requests[slot_req[b]][0].shape[0])
                            self._prefill_slot(s, b, requests[slot_req[b]], pids[slot_req[b]])
                        else:
                            s.finished[b:b + 1].fill_(1)  # idle slot: emits EOS until the session ends
                    while harvests and harvests[0][-1].query():
                        i, hc, hh, hs, hf, _ = harvests.pop(0)
                        if hf is not None and int(hf[0]) != 0:  # never hand out a request decoded on stale partials
                            # the flag is session-wide: every request in flight is suspect -- stop and report them
                            torch.cuda.synchronize(dev)
                            _clear_flags(s)
                            failed = {i} | {h[0] for h in harvests} | {r for r in slot_req if r >= 0}
                            raise HandoffError(failed, queue)
                        # frames [0, F) are final: F = the first EOS in cb0 (within the row's frame range), else the
                        # row's frame count (max_new_tokens - 1)
                        F = min(int(hs[0]), cap_i[i])
                        hit = (hc[:F + 1, 0] == eos).nonzero()
                        F = int(hit[0]) if hit.numel() else F
                        yield i, hc[:F].long(), hh[:F].clone()
                check_handoffs([s])
                self.serve_stats = {"frames": frame, "slots": B, "requests": n}
        finally:
            self.release([s])

    def _prefill_slot(self, s: Session, b: int, req, i: int):
        """Start a request in batch row b (Philox stream id i): per-row state reset, single-request talker prefill into
        row b's K/V (positions 0..P-1, no left padding), first token (M:1746-1800, 2044)."""
        emb, trail = req[0], req[1]
        P, H = int(emb.shape[0]), self.talker.H
        t, dev = self.talker, self.dev
        if P + s.max_frames + 2 > s.Lmax:
            raise ValueError(f"prompt of {P} tokens exceeds the session's K/V capacity ({s.Lmax})")
        for z in (s.seen, s.finished, s.codes):
            z[b].zero_()
        s.prow[b:b + 1].fill_(i)
        s.meta["row_start"][b:b + 1].zero_()
        c = s.ctr.view(5, s.B)
        c[0, b:b + 1].zero_()
        c[1, b:b + 1].fill_(1)
        c[2:4, b:b + 1].fill_(P)
        c[4, b:b + 1].fill_(P + 1)
        tr = s.trailing[b]
        tr.copy_(s.pad_embed.view(1, H).expand_as(tr))
        nt = min(int(trail.shape[0]), tr.shape[0])
        tr[:nt] = trail[:nt].to(dev).float()
        pre = _lru_get(s.slot_prefill, P)
        if pre is None:
            i32 = lambda *z: torch.zeros(*z, dtype=torch.int32, device=dev)  # noqa: E731
            ar = torch.arange(P, device=dev, dtype=torch.int32)
            pre = {"x": torch.empty(P, H, dtype=torch.float32, device=dev), "sc": _scratch(P, t, dev),
                   "meta": {"rope_pos": ar, "kv_pos": ar.clone(), "row_len": ar + 1, "row_start": i32(P),
                            "row_batch": i32(P)},
                   "x16": (torch.empty(P, H, dtype=torch.bfloat16, device=dev)
                           if X16 and self.wdt == torch.bfloat16 and (P <= 96 or PF) else None)}
            _lru_put(s.slot_prefill, P, pre)
        pre["meta"]["row_batch"].fill_(b)
        pre["x"].copy_(emb.reshape(P, H))
        if pre["x16"] is not None:
            pre["x16"].copy_(pre["x"])
        t.forward(pre["x"], P, pre["meta"], s.kv, pre["sc"], s.Lmax, P, x16=pre["x16"])
        K.rmsnorm(pre["x"][P - 1:], t.norm, t.eps, s.past_hidden[b:b + 1], 1, H)
        s.hiddens[b, 0].copy_(s.past_hidden[b])
        K.gemm(s.past_hidden[b:b + 1], self.codec_head, s.logits[b:b + 1], 1, H, self.V)
        self._sample_talker(s, s.logits, 0, 99, b, b + 1)

    def _prefill(self, s: Session, embeds, mask, trailing, tts_pad, seed: int, philox_ids=None):
        """Talker prefill of one row group (M:1746-1800 positions, M:2044 first token) into session s.
        philox_ids: per-row Philox stream ids (default the row index)."""
        B, P, H = embeds.shape
        t = self.talker
        dev = self.dev
        s.P = P  # padded prompt length: every row's decode keys are <= P + frames + 1
        # reset per-request state
        for z in (s.seen, s.finished, s.codes, s.ctr):
            z.zero_()
        s.seed.fill_(seed)
        if philox_ids is None:
            torch.arange(B, dtype=torch.int32, device=dev, out=s.prow)
        else:
            s.prow.copy_(_to_dev_i32(list(philox_ids), dev))
        # stale K/V beyond each row's valid range is never read (row_start/row_len bound every read)
        Ttr = trailing.shape[1]
        s.pad_embed.copy_(tts_pad.reshape(-1).float())
        s.trailing.copy_(s.pad_embed.view(1, 1, H).expand_as(s.trailing))
        n = min(Ttr, s.trailing.shape[1])
        s.trailing[:, :n] = trailing[:, :n].to(dev).float()
        # positions (get_rope_index + rope_deltas, M:1693-1711, 1746-1800)
        mask = mask.to(dev)
        pos = mask.float().cumsum(-1) - 1
        pos = pos.masked_fill(mask == 0, 1)
        max_pos = pos.max(-1)[0]
        n_real = mask.sum(-1)
        n_pads = P - n_real
        rope_delta = (max_pos + 1 - n_real).long() - n_pads
        R = B * P
        pre = _lru_get(s.prefill, P)
        if pre is None:  # static buffers of this prompt length (a captured graph binds their addresses)
            i32 = lambda *z: torch.zeros(*z, dtype=torch.int32, device=dev)  # noqa: E731
            pre = {"x": torch.empty(R, H, dtype=torch.float32, device=dev), "sc": _scratch(R, t, dev),
                   "meta": {"rope_pos": i32(R), "kv_pos": torch.arange(P, device=dev, dtype=torch.int32).repeat(B),
                            "row_len": torch.arange(1, P + 1, device=dev, dtype=torch.int32).repeat(B),
                            "row_start": i32(R),
                            "row_batch": torch.arange(B, device=dev, dtype=torch.int32).repeat_interleave(P)},
                   "last": torch.empty(B, H, dtype=torch.float32, device=dev), "graph": None, "uses": 0,
                   # bf16 shadow of the prefill residual (skinny-GEMV row counts): the RMS GEMVs read half the bytes
                   "x16": (torch.empty(R, H, dtype=torch.bfloat16, device=dev)
                           if X16 and self.wdt == torch.bfloat16 and (R <= 96 or PF) else None)}
            _lru_put(s.prefill, P, pre)
        pre["meta"]["rope_pos"].copy_(pos.reshape(-1))
        pre["meta"]["row_start"].copy_(torch.where(mask.bool(), n_pads[:, None], torch.zeros_like(n_pads)[:, None])
                                       .reshape(-1))
        pre["x"].copy_(embeds.reshape(R, H))
        if pre["graph"] is not None:
            pre["graph"].replay()
        else:
            self._prefill_compute(s, pre, B, P)
            pre["uses"] += 1
            # a prompt length seen twice (streaming-text prompts repeat it: role + codec prefix) gets a captured
            # prefill: ~170 launches replayed instead of issued from Python (host-bound, ~4.6 ms at B=8)
            if PREFILL_GRAPH and pre["uses"] >= 2:
                pre["graph"] = self._capture_prefill(s, pre, B, P)
        # decode counters: step 0, one token generated, pos = P + delta, kv_pos = P, len = P + 1
        s.n_gen.fill_(1)  # a device fill: item assignment uploads a host scalar and waits for the prefill
        s.meta["rope_pos"].copy_((P + rope_delta).to(torch.int32))
        s.meta["kv_pos"].fill_(P)
        s.meta["row_len"].fill_(P + 1)
        s.meta["row_start"].copy_(n_pads.to(torch.int32))

    def _prefill_compute(self, s: Session, pre, B, P):
        """The talker prefill forward over static buffers, then the first token (graph-capturable)."""
        t, H = self.talker, self.talker.H
        if pre["x16"] is not None:
            pre["x16"].copy_(pre["x"])
        t.forward(pre["x"], B * P, pre["meta"], s.kv, pre["sc"], s.Lmax, P, x16=pre["x16"])
        pre["last"].copy_(pre["x"].view(B, P, H)[:, -1])
        K.rmsnorm(pre["last"], t.norm, t.eps, s.past_hidden, B, H)
        K.gemm(s.past_hidden, self.codec_head, s.logits, B, H, self.V)
        self._sample_talker(s, s.logits, 0, 99)

    def _capture_prefill(self, s: Session, pre, B, P):
        snap = s.ctr.clone(), s.seen.clone(), s.finished.clone(), s.codes.clone(), s.tok0.clone(), s.seed.clone()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(side), K.use_workspace(s.ws):
            with torch.cuda.graph(g, stream=side):
                self._prefill_compute(s, pre, B, P)
        torch.cuda.current_stream().wait_stream(side)
        s.ctr.copy_(snap[0]); s.seen.copy_(snap[1]); s.finished.copy_(snap[2]); s.codes.copy_(snap[3])
        s.tok0.copy_(snap[4]); s.seed.copy_(snap[5])
        return g

    def _run_frame(self, s: Session, keys: int, use_graph: bool = True, part: str = "all"):
        """One frame of session s whose rows hold at most `keys` cached talker keys (a host-side bound): the talker
        decode attention's split factor follows the length (attn_nsplit); with graphs, the frame graph of that factor
        is replayed (captured the first time the factor is needed -- a graph binds its launch grids).  part: "all",
        or "cp" / "talk" for a frame issued in two pieces (_frame)."""
        ns = attn_nsplit(keys)
        s.meta["nsplit"] = ns
        if not use_graph:
            self._fence_in()
            with K.use_workspace(s.ws):
                self._frame(s, part)
            self._fence_out()
            return
        g = s.graphs.get((ns, part))
        if g is None:
            g = s.graphs[(ns, part)] = self._capture(s, part)
        if part == "all":
            s.graph = g
        self._fence_in()
        g.replay()
        self._fence_out()

    # Frames of concurrent requests on different streams are serialised on the device: each persistent hand-off kernel
    # of a frame (qt_cp_step / qt_cp_prefill, qt_talker_tail, the head-split attention + o_proj) needs all of its 256
    # workgroups resident at once, one per CU, and two such launches running together could each hold part of the chip
    # while waiting for blocks that cannot start (the bounded polls would then give up and fail both requests).  Each
    # frame waits for the last frame issued on another stream (an event, no host sync); kernels without in-launch
    # hand-offs (codec, prefill) still overlap freely.
    def _fence_in(self):
        cur = torch.cuda.current_stream(self.dev)
        if self._fence is not None and self._fence[1] != cur:
            cur.wait_event(self._fence[0])

    def _fence_out(self):
        cur = torch.cuda.current_stream(self.dev)
        ev = torch.cuda.Event()
        ev.record(cur)
        self._fence = (ev, cur)

    def _capture(self, s: Session, part: str = "all"):
        # the graph must not see the prefill-time counter values: it only reads device memory
        snap = s.ctr.clone(), s.seen.clone(), s.finished.clone(), s.codes.clone(), s.tok0.clone(), s.seed.clone()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(side), K.use_workspace(s.ws):
            with torch.cuda.graph(g, stream=side):
                self._frame(s, part)
        torch.cuda.current_stream().wait_stream(side)
        # capture does not execute kernels on ROCm/CUDA; restore anyway for safety
        s.ctr.copy_(snap[0]); s.seen.copy_(snap[1]); s.finished.copy_(snap[2]); s.codes.copy_(snap[3])
        s.tok0.copy_(snap[4]); s.seed.copy_(snap[5])
        return g
