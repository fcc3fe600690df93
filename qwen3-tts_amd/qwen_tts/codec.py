"""Qwen3-TTS-Tokenizer-12Hz decoder on the MI355X kernels.

Replaces `Qwen3TTSTokenizerV2Decoder.forward / chunked_decode` and `Qwen3TTSTokenizerV2Model.decode`
(K = qwen_tts/core/tokenizer_12hz/modeling_qwen3_tts_tokenizer_v2.py :823-895, 992-1022).
Layout: channels-last [B][T][C] end to end, so every Conv1d / ConvTranspose1d is an implicit GEMM on
the weight-tiled MFMA kernel (transposed convs become 1- or 2-tap convs whose N = stride*Cout output
columns are already the time-interleaved samples: no pixel shuffle pass).
"""
from __future__ import annotations

import math
from typing import Dict, List

import torch

from . import _hip
from . import kernels as K


def _w(W, name, dev):
    t = W[name]
    if not isinstance(t, torch.Tensor):
        t = torch.from_numpy(t)
    return t.to(dev).float()


class CodecDecoder:
    def __init__(self, ccfg: dict, weights: Dict[str, torch.Tensor], dtype="bf16", device="cuda"):
        _hip.lib()
        self.ccfg = ccfg
        self.d = d = ccfg["decoder_config"]
        self.dev = dev = torch.device(device)
        self.wdt = wdt = torch.bfloat16 if dtype == "bf16" else torch.float32
        self.adt = wdt
        W = weights
        g = lambda n: _w(W, n, dev)  # noqa: E731
        # C1: RVQ codebooks (embedding_sum / clamp(cluster_usage)) and the two 1x1 output projections
        Q = d["num_quantizers"]
        tabs = []
        for q in range(Q):
            grp, j = ("rvq_first", q) if q == 0 else ("rvq_rest", q - 1)
            p = f"decoder.quantizer.{grp}.vq.layers.{j}._codebook"
            tabs.append(g(f"{p}.embedding_sum") / g(f"{p}.cluster_usage").clamp(min=1e-5)[:, None])
        self.tables = torch.stack(tabs).contiguous()
        self.cb_dim = self.tables.shape[-1]
        self.proj_first = K.tile_linear(g("decoder.quantizer.rvq_first.output_proj.weight")[:, :, 0], wdt)
        self.proj_rest = K.tile_linear(g("decoder.quantizer.rvq_rest.output_proj.weight")[:, :, 0], wdt)
        # C2
        self.pre_conv = K.tile_conv(g("decoder.pre_conv.conv.weight"), g("decoder.pre_conv.conv.bias"), wdt)
        # C3
        pt = "decoder.pre_transformer"
        self.hid = d["hidden_size"]
        self.heads = d["num_attention_heads"]
        self.kvh = d["num_key_value_heads"]
        self.hd = self.hid // self.heads
        self.inp = K.tile_linear(g(f"{pt}.input_proj.weight"), wdt, g(f"{pt}.input_proj.bias"))
        self.outp = K.tile_linear(g(f"{pt}.output_proj.weight"), wdt, g(f"{pt}.output_proj.bias"), gamma=g(f"{pt}.norm.weight"))
        self.tnorm = g(f"{pt}.norm.weight").contiguous()
        self.layers = []
        for i in range(d["num_hidden_layers"]):
            p = f"{pt}.layers.{i}"
            self.layers.append(dict(
                qkv=K.tile_linear(torch.cat([g(f"{p}.self_attn.q_proj.weight"), g(f"{p}.self_attn.k_proj.weight"),
                                             g(f"{p}.self_attn.v_proj.weight")]), wdt, gamma=g(f"{p}.input_layernorm.weight")),
                o=K.tile_linear(g(f"{p}.self_attn.o_proj.weight"), wdt),
                gu=K.tile_swiglu(g(f"{p}.mlp.gate_proj.weight"), g(f"{p}.mlp.up_proj.weight"), wdt,
                                 gamma=g(f"{p}.post_attention_layernorm.weight")),
                down=K.tile_linear(g(f"{p}.mlp.down_proj.weight"), wdt),
                ln1=g(f"{p}.input_layernorm.weight").contiguous(), ln2=g(f"{p}.post_attention_layernorm.weight").contiguous(),
                ls1=g(f"{p}.self_attn_layer_scale.scale").contiguous(), ls2=g(f"{p}.mlp_layer_scale.scale").contiguous()))
        self.cos, self.sin = K.rope_tables(self.hd, d["rope_theta"], 512, dev)
        # C4
        self.lat = d["latent_dim"]
        self.ups = []
        for i, f in enumerate(d["upsampling_ratios"]):
            p = f"decoder.upsample.{i}"
            self.ups.append(dict(
                f=f, tconv=K.tile_transconv(g(f"{p}.0.conv.weight"), g(f"{p}.0.conv.bias"), wdt, f),
                dw_w=g(f"{p}.1.dwconv.conv.weight")[:, 0, :].contiguous(), dw_b=g(f"{p}.1.dwconv.conv.bias"),
                ln_w=g(f"{p}.1.norm.weight"), ln_b=g(f"{p}.1.norm.bias"),
                pw1=K.tile_linear(g(f"{p}.1.pwconv1.weight"), wdt, g(f"{p}.1.pwconv1.bias")),
                pw2=K.tile_linear(g(f"{p}.1.pwconv2.weight"), wdt, g(f"{p}.1.pwconv2.bias")),
                gamma=g(f"{p}.1.gamma").contiguous()))
        # C5-C7
        self.conv0 = K.tile_conv(g("decoder.decoder.0.conv.weight"), g("decoder.decoder.0.conv.bias"), wdt)
        ds = d["decoder_dim"]
        self.blocks = []
        snake = lambda p: (torch.exp(g(f"{p}.alpha")).contiguous(),  # noqa: E731
                           (1.0 / (torch.exp(g(f"{p}.beta")) + 1e-9)).contiguous())
        for i, r in enumerate(d["upsample_rates"]):
            p = f"decoder.decoder.{i + 1}.block"
            units = []
            for j, dil in enumerate((1, 3, 9)):
                q = f"{p}.{j + 2}"
                units.append(dict(dil=dil, s1=snake(f"{q}.act1"), s2=snake(f"{q}.act2"),
                                  c1=K.tile_conv(g(f"{q}.conv1.conv.weight"), g(f"{q}.conv1.conv.bias"), wdt, dil),
                                  c2=K.tile_conv(g(f"{q}.conv2.conv.weight"), g(f"{q}.conv2.conv.bias"), wdt)))
            self.blocks.append(dict(r=r, cin=ds // 2 ** i, cout=ds // 2 ** (i + 1), s=snake(f"{p}.0"),
                                    tconv=K.tile_transconv(g(f"{p}.1.conv.weight"), g(f"{p}.1.conv.bias"), wdt, r),
                                    units=units))
        n = len(d["upsample_rates"])
        self.c_last = ds // 2 ** n
        self.s_last = snake(f"decoder.decoder.{n + 1}")
        self.conv_last = K.tile_conv(g(f"decoder.decoder.{n + 2}.conv.weight"), g(f"decoder.decoder.{n + 2}.conv.bias"),
                                     wdt)
        self.total_upsample = int(math.prod(d["upsample_rates"]) * math.prod(d["upsampling_ratios"]))
        self._slots = {}  # (B, max_frames) -> [_StreamSlot]: incremental-decode state reused across streams
        torch.cuda.synchronize()

    # ------------------------------------------------------------------------------------------------
    def _conv(self, x, Wt, B, t_in, t_out, t_off, out, cin, epi=_hip.EPI_STORE, act=_hip.ACT_NONE, snake=None):
        K.gemm(x, Wt, out, B * t_out, cin, Wt.N, conv=(t_in, t_out, t_off, getattr(Wt, "dil", 1)), epi=epi, act=act,
               snake=snake)

    def _causal(self, x, Wt, B, T, out, cin, epi=_hip.EPI_STORE, snake=None):
        dil = getattr(Wt, "dil", 1)
        self._conv(x, Wt, B, T, T, -(Wt.taps - 1) * dil, out, cin, epi, snake=snake)

    def _transformer(self, h, B, T):
        """C3 (K:500-574).  h: [B*T][lat] (adt) -> [B*T][lat] (adt)."""
        dev, R = self.dev, B * T
        hid, nh, nkv, D = self.hid, self.heads, self.kvh, self.hd
        x = torch.empty(R, self.inp.N, dtype=torch.float32, device=dev)
        K.gemm(h, self.inp, x, R, self.lat, self.inp.N)
        if self.cos.shape[0] < T:
            self.cos, self.sin = K.rope_tables(D, self.d["rope_theta"], T + 64, dev)
        pos = torch.arange(T, device=dev, dtype=torch.int32).repeat(B)
        meta_b = torch.arange(B, device=dev, dtype=torch.int32).repeat_interleave(T)
        row_len = pos + 1
        row_start = torch.zeros_like(pos)
        qkv_w = (nh + 2 * nkv) * D
        qkv = torch.empty(R, qkv_w, dtype=torch.float32, device=dev)
        q = torch.empty(R, nh * D, dtype=torch.float32, device=dev)
        att = torch.empty(R, nh * D, dtype=torch.float32, device=dev)
        hmid = torch.empty(R, self.d["intermediate_size"], dtype=torch.float32, device=dev)
        kc = torch.empty(B, nkv, T, D, dtype=torch.float32, device=dev)
        vc = torch.empty_like(kc)
        eps, win = self.d["rms_norm_eps"], self.d["sliding_window"]
        for L in self.layers:
            K.gemm(x, L["qkv"], qkv, R, hid, qkv_w, rms=True, eps=eps)
            K.qkv_post(qkv, R, nh, nkv, D, None, None, eps, self.cos, self.sin, pos, meta_b, pos, q, kc, vc, T)
            K.attention(q, R, nh, nkv, D, kc, vc, T, meta_b, row_start, row_len, att, min(win, T), window=win)
            K.gemm(att, L["o"], x, R, nh * D, hid, colscale=L["ls1"], epi=_hip.EPI_ADD)
            K.gemm(x, L["gu"], hmid, R, hid, self.d["intermediate_size"], rms=True, eps=eps, epi=_hip.EPI_SWIGLU)
            K.gemm(hmid, L["down"], x, R, self.d["intermediate_size"], hid, colscale=L["ls2"], epi=_hip.EPI_ADD)
        y = torch.empty(R, self.lat, dtype=self.adt, device=dev)
        K.gemm(x, self.outp, y, R, hid, self.lat, rms=True, eps=eps)
        return y

    def forward(self, codes: torch.Tensor) -> torch.Tensor:
        """codes int [B, T, 16] (device) -> pcm fp32 [B, 1920T-555] (K:868-883)."""
        B, T, Qn = codes.shape
        dev, adt = self.dev, self.adt
        codes = codes.to(dev, torch.int32).contiguous()
        # C1
        o1 = torch.empty(B * T, self.cb_dim, dtype=torch.float32, device=dev)
        o2 = torch.empty_like(o1)
        K.rvq_gather(self.tables, Qn, 1, self.tables.shape[1], self.cb_dim, codes, B, T, o1, o2)
        cd = self.proj_first.N
        h = torch.empty(B * T, cd, dtype=adt, device=dev)
        K.gemm(o1, self.proj_first, h, B * T, self.cb_dim, cd)
        K.gemm(o2, self.proj_rest, h, B * T, self.cb_dim, cd, epi=_hip.EPI_ADD)
        # C2
        x = torch.empty(B * T, self.pre_conv.N, dtype=adt, device=dev)
        self._causal(h, self.pre_conv, B, T, x, cd)
        # C3
        x = self._transformer(x, B, T)
        # C4
        L = T
        C = self.lat
        for u in self.ups:
            f = u["f"]
            y = torch.empty(B * L * f, C, dtype=adt, device=dev)
            self._conv(x, u["tconv"], B, L, L, 0, y, C)
            L *= f
            z = torch.empty_like(y)
            K.dwconv_ln(y, B, L, C, u["dw_w"], u["dw_b"], u["ln_w"], u["ln_b"], 1e-6, z)
            hmid = torch.empty(B * L, u["pw1"].N, dtype=adt, device=dev)
            K.gemm(z, u["pw1"], hmid, B * L, C, u["pw1"].N, act=_hip.ACT_GELU)
            K.gemm(hmid, u["pw2"], y, B * L, u["pw1"].N, C, colscale=u["gamma"], epi=_hip.EPI_ADD)
            x = y
        # C5
        ds = self.d["decoder_dim"]
        y = torch.empty(B * L, self.conv0.N, dtype=adt, device=dev)
        self._causal(x, self.conv0, B, L, y, C)
        x, C = y, ds
        # C6
        # every SnakeBeta feeds a conv: applied to the conv's A operand as it is staged (no separate pass)
        for blk in self.blocks:
            r, cout = blk["r"], blk["cout"]
            Lo = (L - 1) * r
            y = torch.empty(B * Lo, cout, dtype=adt, device=dev)
            self._conv(x, blk["tconv"], B, L, L - 1, 0, y, C, snake=blk["s"])
            L, C, x = Lo, cout, y
            bb = torch.empty_like(x)
            for un in blk["units"]:
                self._causal(x, un["c1"], B, L, bb, C, snake=un["s1"])
                self._causal(bb, un["c2"], B, L, x, C, epi=_hip.EPI_ADD, snake=un["s2"])
        # C7
        out = torch.empty(B * L, self.conv_last.N, dtype=torch.float32, device=dev)
        self._conv(x, self.conv_last, B, L, L, -(self.conv_last.taps - 1), out, C, snake=self.s_last)
        pcm = out[:, 0].contiguous()
        K.clamp_pcm(pcm, pcm.numel(), pcm)
        return pcm.view(B, L)

    def stream(self, B: int, max_frames: int) -> "CodecStream":
        """A stateful incremental decode of up to max_frames frames (one reference chunk with its context); close() it
        to return its state slot (and the slot's captured feed graphs) to the pool."""
        return CodecStream(self, B, max_frames)

    def _acquire_slot(self, B, max_frames) -> "_StreamSlot":
        pool = self._slots.setdefault((B, max_frames), [])
        for sl in pool:
            if not sl.busy:
                sl.reset()
                sl.busy = True
                return sl
        sl = _StreamSlot(self, B, max_frames)
        sl.busy = True
        pool.append(sl)
        return sl

    def chunked_decode(self, codes: torch.Tensor, chunk_size=300, left_context_size=25) -> torch.Tensor:
        """K:885-895 (codes [B, T, 16]; same chunk / left-context semantics, including the >300 quirks)."""
        wavs, start, T = [], 0, codes.shape[1]
        while start < T:
            end = min(start + chunk_size, T)
            ctx = left_context_size if start - left_context_size > 0 else start
            w = self.forward(codes[:, start - ctx:end])
            wavs.append(w[:, ctx * self.total_upsample:])
            start = end
        return torch.cat(wavs, -1)

    def decode(self, audio_codes: torch.Tensor) -> List[torch.Tensor]:
        """Qwen3TTSTokenizerV2Model.decode (K:992-1022): [B, T, 16] -> list of 1-D fp32 wavs (device)."""
        cb = self.tables.shape[1]
        if audio_codes.numel() and (int(audio_codes.min()) < 0 or int(audio_codes.max()) >= cb):
            # the reference's codebook lookup raises on such ids (nn.Embedding / F.embedding IndexError)
            raise ValueError(f"audio codes must lie in [0, {cb}); got [{int(audio_codes.min())}, "
                             f"{int(audio_codes.max())}]")
        if audio_codes.shape[1] == 0:
            return [torch.zeros(0, device=self.dev) for _ in range(audio_codes.shape[0])]
        wav = self.chunked_decode(audio_codes)
        lengths = (audio_codes[..., 0] > 0).sum(1) * self.ccfg["decode_upsample_rate"]
        return [a[:int(l)] for a, l in zip(wav, lengths)]


class _StreamSlot:
    """State of one incremental decode, reused by successive CodecStreams of the same (B, max_frames): the K/V caches,
    every stage's input history (updated in place, so captured graphs keep pointing at it), the frame counter as a
    device word, and the feed graphs captured on this slot keyed by (frames per feed, first feed)."""

    def __init__(self, dec: "CodecDecoder", B: int, max_frames: int):
        dev = dec.dev
        self.kc = [torch.zeros(B, dec.kvh, max_frames, dec.hd, dtype=torch.float32, device=dev) for _ in dec.layers]
        self.vc = [torch.zeros_like(k) for k in self.kc]
        self.nf_dev = torch.zeros(1, dtype=torch.int32, device=dev)
        self.hist = {}      # stage key -> [B][rows][C]
        self.graphs = {}    # (n, first) -> (graph, static codes input, static pcm output)
        self.uses = {}
        self.busy = False
        # split-K scratch of this slot's GEMVs: every feed of the slot (eager or captured) uses it, whatever stream
        # or workspace context the caller is in, so a captured feed graph never points at a caller's temporary
        self.ws = K.new_workspace(dev)

    def reset(self):
        for h in self.hist.values():
            h.zero_()
        self.nf_dev.zero_()


# captured feed graphs (per slot and feed shape, once a shape repeats); QT_CODEC_GRAPH=0 always feeds eagerly (A/B)
CODEC_GRAPH = _hip.lib_knob("QT_CODEC_GRAPH", 1) != 0


class CodecStream:
    """Stateful incremental form of CodecDecoder.forward: frames are fed as they are generated and
    every output sample is computed once.  After n frames have been fed, samples [0, 1920 n - 555) of
    forward(all n frames) are available -- the same prefix, since every stage only looks back (causal convs,
    sliding-window attention) except the decoder blocks' transposed convs, whose output row t needs input rows t and
    t + 1 (their one-row lookahead is what the 555-sample tail is).  State per stage: the last (taps - 1) x dil input
    rows of every causal conv (zeros at the start = the one-shot zero padding), the last input row of every 2-tap
    transposed conv, the transformer's K/V caches (positions 0.. of this decode, window 72).  The per-row math is
    the one-shot's; only the GEMM row counts differ (results equal up to fp summation order).
    A feed of ~140 small launches is host-bound, so a feed shape seen twice on a state slot is captured into a HIP
    graph (positions come from the slot's device frame counter, histories are updated in place) and replayed.
    close() hands the slot back to the decoder's pool.
    """

    def __init__(self, dec: "CodecDecoder", B: int, max_frames: int):
        self.dec, self.B, self.max_frames = dec, B, max_frames
        d = dec.d
        if dec.cos.shape[0] < max_frames:  # old tables stay alive: other slots' captured feed graphs read them
            dec._old_rope = getattr(dec, "_old_rope", []) + [(dec.cos, dec.sin)]
            dec.cos, dec.sin = K.rope_tables(dec.hd, d["rope_theta"], max_frames + 64, dec.dev)
        self.slot = dec._acquire_slot(B, max_frames)
        self.nf = 0  # frames fed
        self.pcm = torch.zeros(B, dec.total_upsample * max_frames, dtype=torch.float32, device=dec.dev)
        self.ns = 0  # valid samples in self.pcm

    def close(self):
        if self.slot is not None:
            self.slot.busy = False
            self.slot = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- stages ----------------------------------------------------------------------------------------
    def _hist(self, key, rows, C, dtype):
        h = self.slot.hist.get(key)
        if h is None:  # first use on this slot (eager, never inside a capture): zeros = the one-shot zero padding
            h = self.slot.hist[key] = torch.zeros(self.B, rows, C, dtype=dtype, device=self.dec.dev)
        return h

    def _causal(self, key, x, n, Wt, cin, out=None, epi=_hip.EPI_STORE, snake=None):
        """x [B][n][cin] new input rows -> [B][n][Wt.N] outputs of the causal conv (history = previous inputs)."""
        dec, B = self.dec, self.B
        H = (Wt.taps - 1) * getattr(Wt, "dil", 1)
        if H:
            h = self._hist(key, H, cin, x.dtype)
            xin = torch.cat([h, x.view(B, n, cin)], 1)
            h.copy_(xin[:, -H:])
        else:
            xin = x
        if out is None:
            out = torch.empty(B * n, Wt.N, dtype=dec.adt, device=dec.dev)
        dec._conv(xin, Wt, B, H + n, n, 0, out, cin, epi=epi, snake=snake)
        return out

    def _tconv2(self, key, x, n, Wt, cin, snake, first):
        """2-tap transposed conv (row t <- inputs t, t + 1): returns (rows out, [B*rows][Wt.N])."""
        dec, B = self.dec, self.B
        h = self._hist(key, 1, cin, x.dtype)
        xin = x.view(B, n, cin) if first else torch.cat([h, x.view(B, n, cin)], 1)
        xin = xin.contiguous()
        L = xin.shape[1]
        h.copy_(xin[:, -1:])
        rows = L - 1
        out = torch.empty(B * max(rows, 0), Wt.N, dtype=dec.adt, device=dec.dev)
        if rows > 0:
            dec._conv(xin, Wt, B, L, rows, 0, out, cin, snake=snake)
        return rows, out

    def _transformer(self, h, n):
        dec, B, dev = self.dec, self.B, self.dec.dev
        R = B * n
        hid, nh, nkv, D = dec.hid, dec.heads, dec.kvh, dec.hd
        x = torch.empty(R, dec.inp.N, dtype=torch.float32, device=dev)
        K.gemm(h, dec.inp, x, R, dec.lat, dec.inp.N)
        # positions nf .. nf + n - 1 from the slot's device frame counter (a captured feed replays with later ones)
        pos = (torch.arange(n, device=dev, dtype=torch.int32) + self.slot.nf_dev).repeat(B)
        meta_b = torch.arange(B, device=dev, dtype=torch.int32).repeat_interleave(n)
        row_len, row_start = pos + 1, torch.zeros_like(pos)
        qkv_w = (nh + 2 * nkv) * D
        qkv = torch.empty(R, qkv_w, dtype=torch.float32, device=dev)
        q = torch.empty(R, nh * D, dtype=torch.float32, device=dev)
        att = torch.empty(R, nh * D, dtype=torch.float32, device=dev)
        inter = dec.d["intermediate_size"]
        hmid = torch.empty(R, inter, dtype=torch.float32, device=dev)
        eps, win, Lm = dec.d["rms_norm_eps"], dec.d["sliding_window"], self.max_frames
        for L, kc, vc in zip(dec.layers, self.slot.kc, self.slot.vc):
            K.gemm(x, L["qkv"], qkv, R, hid, qkv_w, rms=True, eps=eps)
            K.qkv_post(qkv, R, nh, nkv, D, None, None, eps, dec.cos, dec.sin, pos, meta_b, pos, q, kc, vc, Lm)
            K.attention(q, R, nh, nkv, D, kc, vc, Lm, meta_b, row_start, row_len, att, win, window=win)
            K.gemm(att, L["o"], x, R, nh * D, hid, colscale=L["ls1"], epi=_hip.EPI_ADD)
            K.gemm(x, L["gu"], hmid, R, hid, inter, rms=True, eps=eps, epi=_hip.EPI_SWIGLU)
            K.gemm(hmid, L["down"], x, R, inter, hid, colscale=L["ls2"], epi=_hip.EPI_ADD)
        y = torch.empty(R, dec.lat, dtype=dec.adt, device=dev)
        K.gemm(x, dec.outp, y, R, hid, dec.lat, rms=True, eps=eps)
        return y

    # -- feeding ---------------------------------------------------------------------------------------
    def _compute(self, codes: torch.Tensor, n: int, first: bool):
        """The device work of one feed (graph-capturable: no host-side state, fixed shapes for (n, first)); returns
        the new clamped PCM rows [B][L]."""
        dec, B, dev, adt = self.dec, self.B, self.dec.dev, self.dec.adt
        # C1 (per frame)
        o1 = torch.empty(B * n, dec.cb_dim, dtype=torch.float32, device=dev)
        o2 = torch.empty_like(o1)
        K.rvq_gather(dec.tables, codes.shape[2], 1, dec.tables.shape[1], dec.cb_dim, codes, B, n, o1, o2)
        cd = dec.proj_first.N
        h = torch.empty(B * n, cd, dtype=adt, device=dev)
        K.gemm(o1, dec.proj_first, h, B * n, dec.cb_dim, cd)
        K.gemm(o2, dec.proj_rest, h, B * n, dec.cb_dim, cd, epi=_hip.EPI_ADD)
        # C2, C3
        x = self._causal("pre", h, n, dec.pre_conv, cd)
        x = self._transformer(x, n)
        self.slot.nf_dev.add_(n)
        # C4: upsample (1-tap transposed conv, no state) + ConvNeXt (causal depthwise k=7 + LayerNorm, then per row)
        L, C = n, dec.lat
        for i, u in enumerate(dec.ups):
            f = u["f"]
            y = torch.empty(B * L * f, C, dtype=adt, device=dev)
            dec._conv(x, u["tconv"], B, L, L, 0, y, C)
            L *= f
            Hd = u["dw_w"].shape[1] - 1
            hst = self._hist(f"dw{i}", Hd, C, adt)
            yin = torch.cat([hst, y.view(B, L, C)], 1)
            hst.copy_(yin[:, -Hd:])
            z = torch.empty_like(yin)
            K.dwconv_ln(yin, B, Hd + L, C, u["dw_w"], u["dw_b"], u["ln_w"], u["ln_b"], 1e-6, z)
            z = z[:, Hd:].contiguous()
            hmid = torch.empty(B * L, u["pw1"].N, dtype=adt, device=dev)
            K.gemm(z, u["pw1"], hmid, B * L, C, u["pw1"].N, act=_hip.ACT_GELU)
            K.gemm(hmid, u["pw2"], y, B * L, u["pw1"].N, C, colscale=u["gamma"], epi=_hip.EPI_ADD)
            x = y
        # C5
        x = self._causal("conv0", x, L, dec.conv0, C)
        C = dec.d["decoder_dim"]
        # C6
        for bi, blk in enumerate(dec.blocks):
            r, cout = blk["r"], blk["cout"]
            rows, y = self._tconv2(f"t{bi}", x, L, blk["tconv"], C, blk["s"], first)
            L, C, x = rows * r, cout, y
            if L == 0:
                return torch.zeros(B, 0, dtype=torch.float32, device=dev)
            for ui, un in enumerate(blk["units"]):
                bb = self._causal(f"u{bi}.{ui}", x, L, un["c1"], C, snake=un["s1"])
                self._causal(f"v{bi}.{ui}", bb, L, un["c2"], C, out=x, epi=_hip.EPI_ADD, snake=un["s2"])
        # C7
        out = self._causal("last", x, L, dec.conv_last, C, out=torch.empty(B * L, dec.conv_last.N, dtype=torch.float32,
                                                                            device=dev), snake=dec.s_last)
        pcm = out[:, 0].contiguous()
        K.clamp_pcm(pcm, pcm.numel(), pcm)
        return pcm.view(B, L)

    def feed(self, codes: torch.Tensor) -> int:
        """codes int [B, n, 16] (the next n frames) -> number of valid samples now in self.pcm."""
        dec, B, dev = self.dec, self.B, self.dec.dev
        n = codes.shape[1]
        if n == 0:
            return self.ns
        if self.nf + n > self.max_frames:
            raise ValueError(f"CodecStream holds {self.max_frames} frames; {self.nf} fed, {n} more given")
        codes = codes.to(dev, torch.int32).contiguous()
        key = (n, self.nf == 0)
        slot = self.slot
        g = slot.graphs.get(key)
        if g is not None:
            g[1].copy_(codes)
            g[0].replay()
            pcm = g[2]
        else:
            with K.use_workspace(slot.ws):
                pcm = self._compute(codes, n, key[1])
                slot.uses[key] = slot.uses.get(key, 0) + 1
                if CODEC_GRAPH and slot.uses[key] >= 2:
                    slot.graphs[key] = self._capture(codes, n, key[1])
        self.nf += n
        L = pcm.shape[1]
        self.pcm[:, self.ns:self.ns + L] = pcm
        self.ns += L
        return self.ns

    def _capture(self, codes, n, first):
        # capturing executes nothing: the slot state (histories, caches, frame counter) is left as the eager feed left it
        cin = codes.clone()
        side = torch.cuda.Stream(device=self.dec.dev)
        side.wait_stream(torch.cuda.current_stream(self.dec.dev))
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(side):
            with torch.cuda.graph(g, stream=side):
                out = self._compute(cin, n, first)
        torch.cuda.current_stream(self.dec.dev).wait_stream(side)
        return g, cin, out
