"""12 Hz tokenizer ENCODER on the MI355X kernels (voice-clone front end).

Replaces `Qwen3TTSTokenizerV2Model.encode` (K = qwen_tts/core/tokenizer_12hz/modeling_qwen3_tts_tokenizer_v2.py
:960-990), whose body is transformers' `MimiModel.encode` (T = transformers models/mimi/modeling_mimi.py):
SEANet conv stack (T:450-492) -> 8-layer sliding-window transformer (T:729-929) -> stride-2 downsample conv
(T:1205-1214) -> split residual VQ (T:1084-1127), keeping `encoder_valid_num_quantizers` codebooks.

Layout: channels-last [B][T][C] throughout, fp32 activations, weights bf16 or fp32 in MFMA tiles.
* Every strided conv (kernel 2r, stride r) is a 2-tap conv over the *polyphase view* of its input: a
  [B][Tp][C] buffer read as [B][Tp/r][r*C] (a free reshape), so the MFMA implicit GEMM runs at stride 1
  with K = 2*r*C.  The first conv (1 input channel, k=7) is the same trick the other way round: the
  [B][Tp] waveform is read as [B][Tp/8][8] and the conv emits 8 time-interleaved outputs per row.
* Buffers are sized for Tp0 = 960 * ceil(L / 960) samples, so every level's length is a whole number of
  strides.  MimiConv1d's right "extra" zero padding (T:269-279) is reproduced by zeroing rows past the
  level's valid length right before each strided conv (causal convs never look right, so nothing else
  reads those rows).
* The ELU in front of every encoder conv is applied to the GEMM's A operand as it is loaded (QT_AACT_ELU).
* Nearest-codeword search: per codebook stage one launch over (codeword slice x frame tile) blocks, exact fp32
  distances, deterministic last-arriver reduction (qt_rvq_encode).
"""
from __future__ import annotations

import math
from typing import Dict, List

import torch

from . import _hip
from . import kernels as K


def mimi_config(ccfg: dict) -> dict:
    """MimiConfig defaults (transformers configuration_mimi.py) overlaid with the checkpoint's encoder_config."""
    c = dict(sampling_rate=24000, audio_channels=1, hidden_size=512, num_filters=64, num_residual_layers=1,
             upsampling_ratios=[8, 6, 5, 4], kernel_size=7, last_kernel_size=3, residual_kernel_size=3,
             dilation_growth_rate=2, use_causal_conv=True, pad_mode="constant", compress=2, codebook_size=2048,
             codebook_dim=None, num_quantizers=32, use_conv_shortcut=False, vector_quantization_hidden_dimension=256,
             num_semantic_quantizers=1, num_hidden_layers=8, intermediate_size=2048, num_attention_heads=8,
             num_key_value_heads=8, head_dim=None, hidden_act="gelu", norm_eps=1e-5, sliding_window=250,
             layer_scale_initial_scale=0.01, attention_bias=False, rope_theta=10000.0)
    c.update(ccfg.get("encoder_config", {}) or {})
    rp = c.get("rope_parameters") or {}
    if "rope_theta" in rp:
        c["rope_theta"] = rp["rope_theta"]
    if c["codebook_dim"] is None:
        c["codebook_dim"] = c["hidden_size"]
    if not c["head_dim"]:
        c["head_dim"] = c["hidden_size"] // c["num_attention_heads"]
    if (not c["use_causal_conv"] or c["num_residual_layers"] != 1 or c["use_conv_shortcut"] or c["audio_channels"] != 1
            or c["pad_mode"] != "constant" or c["hidden_act"] != "gelu" or c["attention_bias"]):
        raise NotImplementedError("unsupported tokenizer encoder configuration for the MI355X encoder")
    return c


def encoder_specs(ccfg: dict):
    """(name, shape) of the encoder parameters in speech_tokenizer/model.safetensors (prefix `encoder.`)."""
    c = mimi_config(ccfg)
    nf, H = c["num_filters"], c["hidden_size"]
    s = [("encoder.encoder.layers.0.conv.weight", (nf, 1, c["kernel_size"])), ("encoder.encoder.layers.0.conv.bias", (nf,))]
    li, scale = 1, 1
    for r in reversed(c["upsampling_ratios"]):
        C = nf * scale
        hid = C // c["compress"]
        s += [(f"encoder.encoder.layers.{li}.block.1.conv.weight", (hid, C, c["residual_kernel_size"])),
              (f"encoder.encoder.layers.{li}.block.1.conv.bias", (hid,)),
              (f"encoder.encoder.layers.{li}.block.3.conv.weight", (C, hid, 1)),
              (f"encoder.encoder.layers.{li}.block.3.conv.bias", (C,)),
              (f"encoder.encoder.layers.{li + 2}.conv.weight", (2 * C, C, 2 * r)),
              (f"encoder.encoder.layers.{li + 2}.conv.bias", (2 * C,))]
        li += 3
        scale *= 2
    s += [(f"encoder.encoder.layers.{li + 1}.conv.weight", (H, nf * scale, c["last_kernel_size"])),
          (f"encoder.encoder.layers.{li + 1}.conv.bias", (H,))]
    hd, nh, kv, I = c["head_dim"], c["num_attention_heads"], c["num_key_value_heads"], c["intermediate_size"]
    for i in range(c["num_hidden_layers"]):
        p = f"encoder.encoder_transformer.layers.{i}"
        s += [(f"{p}.self_attn.q_proj.weight", (nh * hd, H)), (f"{p}.self_attn.k_proj.weight", (kv * hd, H)),
              (f"{p}.self_attn.v_proj.weight", (kv * hd, H)), (f"{p}.self_attn.o_proj.weight", (H, nh * hd)),
              (f"{p}.mlp.fc1.weight", (I, H)), (f"{p}.mlp.fc2.weight", (H, I)),
              (f"{p}.input_layernorm.weight", (H,)), (f"{p}.input_layernorm.bias", (H,)),
              (f"{p}.post_attention_layernorm.weight", (H,)), (f"{p}.post_attention_layernorm.bias", (H,)),
              (f"{p}.self_attn_layer_scale.scale", (H,)), (f"{p}.mlp_layer_scale.scale", (H,))]
    s += [("encoder.downsample.conv.weight", (H, H, 4))]
    vq, cb, cd, nsem = c["vector_quantization_hidden_dimension"], c["codebook_size"], c["codebook_dim"], \
        c["num_semantic_quantizers"]
    for grp, n in (("semantic_residual_vector_quantizer", nsem),
                   ("acoustic_residual_vector_quantizer", c["num_quantizers"] - nsem)):
        p = f"encoder.quantizer.{grp}"
        s += [(f"{p}.input_proj.weight", (vq, H, 1))]
        for i in range(n):
            s += [(f"{p}.layers.{i}.codebook.cluster_usage", (cb,)), (f"{p}.layers.{i}.codebook.embed_sum", (cb, cd))]
    return s


def _polyphase_weight(w: torch.Tensor, r: int) -> torch.Tensor:
    """Strided conv weight [Cout][Cin][2r] -> 2-tap weight over the polyphase view [Cout][2][r*Cin]:
    W'[o][a][b*Cin + c] = w[o][c][r*a + b] (input row t'-1+a of the view holds samples r(t'-1+a) + b)."""
    co, ci, k = w.shape
    assert k == 2 * r
    return w.reshape(co, ci, 2, r).permute(0, 2, 3, 1).reshape(co, 2, r * ci)


def _first_conv_weight(w: torch.Tensor, P: int) -> torch.Tensor:
    """Causal conv weight [Cout][1][k] (k <= P + 1) -> 2-tap weight over the waveform viewed as [Tp/P][P], emitting
    P time-interleaved outputs per row: W'[phi*Cout + o][a][c] = w[o][0][P*a + c - phi - (P - k + 1)]."""
    co, _, k = w.shape
    out = torch.zeros(P * co, 2, P, dtype=w.dtype, device=w.device)
    for phi in range(P):
        for a in range(2):
            for c in range(P):
                j = P * a + c - phi - (P - k + 1)
                if 0 <= j < k:
                    out[phi * co:(phi + 1) * co, a, c] = w[:, 0, j]
    return out


def _tile_taps(w3: torch.Tensor, b, dtype, cin):
    """[N][taps][cin] -> Tiled implicit-conv weight (cin padded to the MFMA k tile)."""
    N, taps, _ = w3.shape
    wk, cp = K._pad_cin(w3, cin, dtype)
    t = K.tile(wk.reshape(N, taps * cp), dtype, b, taps=taps, cin=cin, cin_pad=cp, K=taps * cp)
    t.dil = 1
    return t


class TokenizerEncoder:
    P0 = 8  # waveform samples per row of the first conv's polyphase view

    def __init__(self, ccfg: dict, weights: Dict[str, torch.Tensor], dtype="bf16", device="cuda"):
        _hip.lib()
        self.ccfg = ccfg
        self.c = c = mimi_config(ccfg)
        self.dev = dev = torch.device(device)
        self.wdt = wdt = torch.bfloat16 if dtype == "bf16" else torch.float32
        g = lambda n: (weights[n] if isinstance(weights[n], torch.Tensor) else torch.from_numpy(weights[n])).to(dev).float()  # noqa: E731
        self.valid_q = int(ccfg.get("encoder_valid_num_quantizers", 16))
        self.down = int(ccfg.get("encode_downsample_rate", 1920))
        self.ratios = list(reversed(c["upsampling_ratios"]))
        self.hop = int(math.prod(self.ratios))
        if c["kernel_size"] > self.P0 + 1:
            raise NotImplementedError("first encoder conv wider than the polyphase view")
        p = "encoder.encoder.layers"
        nf = c["num_filters"]
        w0 = g(f"{p}.0.conv.weight")
        self.conv0 = _tile_taps(_first_conv_weight(w0, self.P0), g(f"{p}.0.conv.bias").repeat(self.P0), wdt, self.P0)
        self.levels = []
        li, C = 1, nf
        wd = lambda cin: wdt if cin % 8 == 0 else torch.float32  # noqa: E731  (bf16 A loads are 8-wide)
        for r in self.ratios:
            self.levels.append(dict(
                r=r, C=C,
                res1=K.tile_conv(g(f"{p}.{li}.block.1.conv.weight"), g(f"{p}.{li}.block.1.conv.bias"), wd(C)),
                res2=K.tile_conv(g(f"{p}.{li}.block.3.conv.weight"), g(f"{p}.{li}.block.3.conv.bias"), wd(C // 2)),
                down=_tile_taps(_polyphase_weight(g(f"{p}.{li + 2}.conv.weight"), r), g(f"{p}.{li + 2}.conv.bias"), wdt,
                                r * C)))
            li += 3
            C *= 2
        self.c_last = C
        self.conv_last = K.tile_conv(g(f"{p}.{li + 1}.conv.weight"), g(f"{p}.{li + 1}.conv.bias"), wdt)
        H = self.H = c["hidden_size"]
        self.nh, self.nkv, self.hd = c["num_attention_heads"], c["num_key_value_heads"], c["head_dim"]
        self.layers = []
        for i in range(c["num_hidden_layers"]):
            q = f"encoder.encoder_transformer.layers.{i}"
            self.layers.append(dict(
                qkv=K.tile_linear(torch.cat([g(f"{q}.self_attn.q_proj.weight"), g(f"{q}.self_attn.k_proj.weight"),
                                             g(f"{q}.self_attn.v_proj.weight")]), wdt),
                o=K.tile_linear(g(f"{q}.self_attn.o_proj.weight"), wdt),
                fc1=K.tile_linear(g(f"{q}.mlp.fc1.weight"), wdt), fc2=K.tile_linear(g(f"{q}.mlp.fc2.weight"), wdt),
                ln1=(g(f"{q}.input_layernorm.weight").contiguous(), g(f"{q}.input_layernorm.bias").contiguous()),
                ln2=(g(f"{q}.post_attention_layernorm.weight").contiguous(),
                     g(f"{q}.post_attention_layernorm.bias").contiguous()),
                ls1=g(f"{q}.self_attn_layer_scale.scale").contiguous(), ls2=g(f"{q}.mlp_layer_scale.scale").contiguous()))
        self.cos, self.sin = K.rope_tables(self.hd, c["rope_theta"], 512, dev)
        self.downsample = _tile_taps(_polyphase_weight(g("encoder.downsample.conv.weight"), 2), None, wdt, 2 * H)
        # quantizer: both groups' input projections in one GEMM; fp32 codebooks (+ transposed copies)
        nsem = c["num_semantic_quantizers"]
        self.nsem = min(nsem, self.valid_q)
        self.nac = max(0, self.valid_q - nsem)
        if self.valid_q > c["num_quantizers"]:
            raise ValueError("encoder_valid_num_quantizers exceeds the encoder's quantizers")
        qp = "encoder.quantizer"
        self.vq = c["vector_quantization_hidden_dimension"]
        self.in_proj = K.tile_linear(torch.cat([g(f"{qp}.semantic_residual_vector_quantizer.input_proj.weight")[:, :, 0],
                                                g(f"{qp}.acoustic_residual_vector_quantizer.input_proj.weight")[:, :, 0]]),
                                     torch.float32)

        def tables(grp, n):
            if n == 0:
                return None, None
            t = torch.stack([g(f"{qp}.{grp}.layers.{i}.codebook.embed_sum")
                             / g(f"{qp}.{grp}.layers.{i}.codebook.cluster_usage").clamp(min=1e-5)[:, None]
                             for i in range(n)]).contiguous()
            return t, t.transpose(1, 2).contiguous()

        self.tab_s, self.tabT_s = tables("semantic_residual_vector_quantizer", self.nsem)
        self.tab_a, self.tabT_a = tables("acoustic_residual_vector_quantizer", self.nac)
        self.cb, self.cd = c["codebook_size"], c["codebook_dim"]
        torch.cuda.synchronize(dev)

    # ------------------------------------------------------------------------------------------------
    def _transformer(self, x: torch.Tensor, B: int, T: int):
        """MimiTransformerModel (T:801-929) in place on the fp32 residual stream x [B*T][H]."""
        dev, R, H = self.dev, B * T, self.H
        nh, nkv, D = self.nh, self.nkv, self.hd
        if self.cos.shape[0] < T:
            self.cos, self.sin = K.rope_tables(D, self.c["rope_theta"], T + 64, dev)
        pos = torch.arange(T, device=dev, dtype=torch.int32).repeat(B)
        meta_b = torch.arange(B, device=dev, dtype=torch.int32).repeat_interleave(T)
        row_len, row_start = pos + 1, torch.zeros_like(pos)
        qkv_w = (nh + 2 * nkv) * D
        xn = torch.empty(R, H, dtype=torch.float32, device=dev)
        qkv = torch.empty(R, qkv_w, dtype=torch.float32, device=dev)
        q = torch.empty(R, nh * D, dtype=torch.float32, device=dev)
        att = torch.empty(R, nh * D, dtype=torch.float32, device=dev)
        hmid = torch.empty(R, self.c["intermediate_size"], dtype=torch.float32, device=dev)
        kc = torch.empty(B, nkv, T, D, dtype=torch.float32, device=dev)
        vc = torch.empty_like(kc)
        eps, win = self.c["norm_eps"], self.c["sliding_window"]
        I = self.c["intermediate_size"]
        for L in self.layers:
            K.layernorm(x, L["ln1"][0], L["ln1"][1], eps, xn, R, H)
            K.gemm(xn, L["qkv"], qkv, R, H, qkv_w)
            K.qkv_post(qkv, R, nh, nkv, D, None, None, 0.0, self.cos, self.sin, pos, meta_b, pos, q, kc, vc, T)
            K.attention(q, R, nh, nkv, D, kc, vc, T, meta_b, row_start, row_len, att, min(win, T), window=win)
            K.gemm(att, L["o"], x, R, nh * D, H, colscale=L["ls1"], epi=_hip.EPI_ADD)
            K.layernorm(x, L["ln2"][0], L["ln2"][1], eps, xn, R, H)
            K.gemm(xn, L["fc1"], hmid, R, H, I, act=_hip.ACT_GELU)
            K.gemm(hmid, L["fc2"], x, R, I, H, colscale=L["ls2"], epi=_hip.EPI_ADD)

    def embeddings(self, wav: torch.Tensor) -> torch.Tensor:
        """wav fp32 [B, L] (device) -> downsampled embeddings fp32 [B*T12][H] and T12 (T:1230-1262)."""
        B, L = wav.shape
        dev = self.dev
        T25 = -(-L // self.hop)
        Tp = T25 * self.hop
        xin = torch.zeros(B, Tp, dtype=torch.float32, device=dev)
        xin[:, :L] = wav
        # conv0 on the polyphase view [B][Tp/8][8] -> [B][Tp][nf]
        nf = self.c["num_filters"]
        x = torch.empty(B * Tp, nf, dtype=torch.float32, device=dev)
        rows = Tp // self.P0
        K.gemm(xin, self.conv0, x, B * rows, self.P0, self.P0 * nf, conv=(rows, rows, -1, 1))
        v = L  # valid length at this level
        for lv in self.levels:
            r, C = lv["r"], lv["C"]
            h = torch.empty(B * Tp, C // 2, dtype=torch.float32, device=dev)
            K.gemm(x, lv["res1"], h, B * Tp, C, C // 2, conv=(Tp, Tp, -(lv["res1"].taps - 1), 1), a_act=_hip.AACT_ELU)
            K.gemm(h, lv["res2"], x, B * Tp, C // 2, C, conv=(Tp, Tp, 0, 1), a_act=_hip.AACT_ELU, epi=_hip.EPI_ADD)
            K.zero_tail(x, B, Tp, v, C)
            Tn = Tp // r
            y = torch.empty(B * Tn, 2 * C, dtype=torch.float32, device=dev)
            K.gemm(x, lv["down"], y, B * Tn, r * C, 2 * C, conv=(Tn, Tn, -1, 1), a_act=_hip.AACT_ELU)
            x, Tp, v = y, Tn, -(-v // r)
        H = self.H
        h = torch.empty(B * Tp, H, dtype=torch.float32, device=dev)
        K.gemm(x, self.conv_last, h, B * Tp, self.c_last, H, conv=(Tp, Tp, -(self.conv_last.taps - 1), 1),
               a_act=_hip.AACT_ELU)
        self._transformer(h, B, Tp)
        # downsample: replicate-pad (left 2, right to even) then a 2-tap valid conv over the [.., 2H] view
        ext = Tp % 2
        Tq = Tp + 2 + ext
        hp = torch.empty(B * Tq, H, dtype=torch.float32, device=dev)
        K.pad_time(h, B, Tp, H, 2, ext, _hip.PAD_REPLICATE, hp)
        T12 = (Tp + ext) // 2
        e = torch.empty(B * T12, H, dtype=torch.float32, device=dev)
        K.gemm(hp, self.downsample, e, B * T12, 2 * H, H, conv=(Tq // 2, T12, 0, 1))
        return e, T12

    def quantize(self, e: torch.Tensor, R: int) -> torch.Tensor:
        """MimiSplitResidualVectorQuantizer.encode for the first valid_q codebooks: [R][H] -> int32 [R][valid_q]."""
        vq = self.vq
        proj = torch.empty(R, 2 * vq, dtype=torch.float32, device=self.dev)
        K.gemm(e, self.in_proj, proj, R, self.H, 2 * vq)
        codes = torch.empty(R, self.valid_q, dtype=torch.int32, device=self.dev)
        if self.nsem:
            K.rvq_encode(proj, 2 * vq, self.tab_s, self.tabT_s, self.nsem, self.cb, self.cd, R, codes, self.valid_q)
        if self.nac:
            K.rvq_encode(proj[:, vq:], 2 * vq, self.tab_a, self.tabT_a, self.nac, self.cb, self.cd, R,
                         codes[:, self.nsem:], self.valid_q)
        return codes

    def encode(self, wavs: List[torch.Tensor]) -> List[torch.Tensor]:
        """Right zero-pad the batch (EncodecFeatureExtractor), encode, keep ceil(len / 1920) frames per item
        (K:983): list of int64 [T_i, valid_q] device tensors."""
        lens = [int(w.shape[0]) for w in wavs]
        if not lens or max(lens) == 0:
            return [torch.zeros(0, self.valid_q, dtype=torch.long, device=self.dev) for _ in lens]
        L = max(lens)
        x = torch.zeros(len(wavs), L, dtype=torch.float32, device=self.dev)
        for i, w in enumerate(wavs):
            x[i, : lens[i]] = w.to(self.dev, torch.float32)
        e, T12 = self.embeddings(x)
        codes = self.quantize(e, len(wavs) * T12).view(len(wavs), T12, self.valid_q)
        return [codes[i, : -(-n // self.down)].long() for i, n in enumerate(lens)]
