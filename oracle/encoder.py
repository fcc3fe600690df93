"""CPU fp32 restatement of the 12 Hz tokenizer ENCODER (voice-clone front end).

TEST INFRASTRUCTURE (oracle/): parity checker for the HIP encoder path; never imported by the product.

The reference's encoder is transformers' `MimiModel` (K = qwen_tts/core/tokenizer_12hz/
modeling_qwen3_tts_tokenizer_v2.py:898-907 subclasses it and drops the decoder half; K:960-990 calls
`encode` and keeps the first `encoder_valid_num_quantizers` codebooks).  The Mimi arithmetic therefore
lives in a third-party dependency: transformers==4.57.3 is pinned (pyproject.toml:24), this image ships
5.15.0, whose `models/mimi/modeling_mimi.py` is what the golden fixtures were generated with
(tests/golden/make_golden.py, `frontend` fixtures).  Restated here (T = that file):
  MimiConv1d (T:210-347): causal left pad (k-1)*d - (s-1)... = k_eff - stride, right "extra" pad to a
      whole number of strides, pad mode constant (replicate for the downsample conv)
  MimiResnetBlock (T:408-447): ELU -> conv k3 (C -> C/2) -> ELU -> conv k1 (C/2 -> C), identity shortcut
  MimiEncoder (T:450-492): conv k7 -> [resblock, ELU, strided conv (k = 2r, stride r)] x r in (4, 5, 6, 8)
      -> ELU -> conv k3 (-> hidden)
  MimiTransformerModel (T:729-929): LayerNorm -> attention (RoPE, causal, sliding window) -> LayerScale ->
      residual; LayerNorm -> fc1 -> GELU -> fc2 -> LayerScale -> residual; no final norm
  downsample (T:1205-1214): MimiConv1d k=4 stride 2, no bias, replicate padding
  MimiSplitResidualVectorQuantizer.encode (T:1084-1127), MimiResidualVectorQuantizer.encode (T:1050-1068),
      MimiEuclideanCodebook (T:964-1007): input_proj 1x1 conv per group, nearest codeword (cdist argmin,
      first index on ties), residual -= codeword
Layout here is channels-first [B, C, T] like the reference.
"""
from __future__ import annotations

import math
from typing import Dict, List

import torch
import torch.nn.functional as F

Tensor = torch.Tensor


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
    if not c["use_causal_conv"] or c["num_residual_layers"] != 1 or c["use_conv_shortcut"] or c["audio_channels"] != 1:
        raise NotImplementedError("only the causal, 1-residual-layer, mono Mimi encoder of Qwen3-TTS is restated")
    return c


def encoder_param_specs(ccfg: dict):
    """(name, shape) of every encoder parameter as stored in speech_tokenizer/model.safetensors
    (`encoder.` = Qwen3TTSTokenizerV2Model.encoder, K:952)."""
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
              (f"encoder.encoder.layers.{li}.block.3.conv.bias", (C,))]
        s += [(f"encoder.encoder.layers.{li + 2}.conv.weight", (2 * C, C, 2 * r)),
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
    vq, cb, cd = c["vector_quantization_hidden_dimension"], c["codebook_size"], c["codebook_dim"]
    nsem = c["num_semantic_quantizers"]
    for grp, n in (("semantic_residual_vector_quantizer", nsem),
                   ("acoustic_residual_vector_quantizer", c["num_quantizers"] - nsem)):
        p = f"encoder.quantizer.{grp}"
        s += [(f"{p}.input_proj.weight", (vq, H, 1)), (f"{p}.output_proj.weight", (H, vq, 1))]
        for i in range(n):
            s += [(f"{p}.layers.{i}.codebook.initialized", (1,)), (f"{p}.layers.{i}.codebook.cluster_usage", (cb,)),
                  (f"{p}.layers.{i}.codebook.embed_sum", (cb, cd))]
    return s


def mimi_conv(x: Tensor, w: Tensor, b, stride=1, dilation=1, pad_mode="constant") -> Tensor:
    """MimiConv1d.forward, causal branch (T:327-347, _get_extra_padding_for_conv1d T:269-279)."""
    k_eff = (w.shape[-1] - 1) * dilation + 1
    pad_total = k_eff - stride
    L = x.shape[-1]
    n_frames = math.ceil((L - k_eff + pad_total) / stride + 1) - 1
    extra = n_frames * stride + k_eff - pad_total - L
    x = F.pad(x, (pad_total, extra), mode=pad_mode)
    return F.conv1d(x, w, b, stride=stride, dilation=dilation)


def layer_norm(x: Tensor, w: Tensor, b: Tensor, eps: float) -> Tensor:
    return F.layer_norm(x, (x.shape[-1],), w, b, eps)


def rope(x: Tensor, theta: float) -> Tensor:
    """rotate-half RoPE at positions 0..T-1 (MimiRotaryEmbedding T:511-560, apply_rotary_pos_emb T:570-600);
    x [B, heads, T, hd]."""
    hd, T = x.shape[-1], x.shape[-2]
    inv = 1.0 / (theta ** (torch.arange(0, hd, 2, dtype=torch.float) / hd))
    fr = torch.arange(T, dtype=torch.float)[:, None] * inv[None, :]
    emb = torch.cat([fr, fr], -1)
    cos, sin = emb.cos(), emb.sin()
    x1, x2 = x[..., : hd // 2], x[..., hd // 2:]
    return x * cos + torch.cat([-x2, x1], -1) * sin


class EncoderOracle:
    """Qwen3TTSTokenizerV2Model.encode (K:960-990) on fp32 CPU tensors keyed by checkpoint names."""

    def __init__(self, ccfg: dict, weights: Dict[str, Tensor]):
        self.c = mimi_config(ccfg)
        self.W = {k: (v if isinstance(v, torch.Tensor) else torch.from_numpy(v)).float() for k, v in weights.items()
                  if k.startswith("encoder.")}
        self.valid_q = int(ccfg.get("encoder_valid_num_quantizers", 16))
        self.down = int(ccfg.get("encode_downsample_rate", 1920))

    def seanet(self, x: Tensor) -> Tensor:
        """MimiEncoder.forward (T:486-492); x [B, 1, L] -> [B, hidden, T25]."""
        c, W = self.c, self.W
        p = "encoder.encoder.layers"
        x = mimi_conv(x, W[f"{p}.0.conv.weight"], W[f"{p}.0.conv.bias"])
        li = 1
        for r in reversed(c["upsampling_ratios"]):
            h = mimi_conv(F.elu(x), W[f"{p}.{li}.block.1.conv.weight"], W[f"{p}.{li}.block.1.conv.bias"])
            h = mimi_conv(F.elu(h), W[f"{p}.{li}.block.3.conv.weight"], W[f"{p}.{li}.block.3.conv.bias"])
            x = x + h
            x = mimi_conv(F.elu(x), W[f"{p}.{li + 2}.conv.weight"], W[f"{p}.{li + 2}.conv.bias"], stride=r)
            li += 3
        return mimi_conv(F.elu(x), W[f"{p}.{li + 1}.conv.weight"], W[f"{p}.{li + 1}.conv.bias"])

    def transformer(self, h: Tensor) -> Tensor:
        """MimiTransformerModel.forward (T:801-929); h [B, T, hidden]."""
        c, W = self.c, self.W
        B, T, H = h.shape
        nh, kv, hd = c["num_attention_heads"], c["num_key_value_heads"], c["head_dim"]
        q_idx = torch.arange(T)[:, None]
        k_idx = torch.arange(T)[None, :]
        allowed = (k_idx <= q_idx) & (k_idx > q_idx - c["sliding_window"])
        for i in range(c["num_hidden_layers"]):
            p = f"encoder.encoder_transformer.layers.{i}"
            x = layer_norm(h, W[f"{p}.input_layernorm.weight"], W[f"{p}.input_layernorm.bias"], c["norm_eps"])
            q = (x @ W[f"{p}.self_attn.q_proj.weight"].T).view(B, T, nh, hd).transpose(1, 2)
            k = (x @ W[f"{p}.self_attn.k_proj.weight"].T).view(B, T, kv, hd).transpose(1, 2)
            v = (x @ W[f"{p}.self_attn.v_proj.weight"].T).view(B, T, kv, hd).transpose(1, 2)
            q, k = rope(q, c["rope_theta"]), rope(k, c["rope_theta"])
            if nh != kv:
                k = k.repeat_interleave(nh // kv, 1)
                v = v.repeat_interleave(nh // kv, 1)
            s = (q @ k.transpose(2, 3)) / math.sqrt(hd)
            s = s.masked_fill(~allowed, float("-inf"))
            a = torch.softmax(s, -1) @ v
            a = a.transpose(1, 2).reshape(B, T, nh * hd) @ W[f"{p}.self_attn.o_proj.weight"].T
            h = h + W[f"{p}.self_attn_layer_scale.scale"] * a
            x = layer_norm(h, W[f"{p}.post_attention_layernorm.weight"], W[f"{p}.post_attention_layernorm.bias"],
                           c["norm_eps"])
            m = F.gelu(x @ W[f"{p}.mlp.fc1.weight"].T) @ W[f"{p}.mlp.fc2.weight"].T
            h = h + W[f"{p}.mlp_layer_scale.scale"] * m
        return h

    def codebook(self, grp: str, i: int) -> Tensor:
        p = f"encoder.quantizer.{grp}.layers.{i}.codebook"
        return self.W[f"{p}.embed_sum"] / self.W[f"{p}.cluster_usage"].clamp(min=1e-5)[:, None]

    def quantize(self, emb: Tensor, nq: int) -> Tensor:
        """MimiSplitResidualVectorQuantizer.encode for the first nq codebooks; emb [B, hidden, T12] -> [B, nq, T12].
        Distances in float64 (the nearest codeword; the reference's cdist is fp32, see margins())."""
        c = self.c
        nsem = c["num_semantic_quantizers"]
        out = []
        for grp, n in (("semantic_residual_vector_quantizer", min(nsem, nq)),
                       ("acoustic_residual_vector_quantizer", max(0, nq - nsem))):
            if n == 0:
                continue
            r = F.conv1d(emb, self.W[f"encoder.quantizer.{grp}.input_proj.weight"]).transpose(1, 2).double()
            for i in range(n):
                e = self.codebook(grp, i).double()
                d = ((r[:, :, None, :] - e[None, None]) ** 2).sum(-1)  # [B, T, cb]
                idx = d.argmin(-1)
                out.append(idx)
                r = r - e[idx]
        return torch.stack(out, 1)

    def margins(self, emb: Tensor, nq: int) -> Tensor:
        """(second-best - best) / best squared distance per (b, q, t): how far each choice is from a tie."""
        c = self.c
        nsem = c["num_semantic_quantizers"]
        out = []
        for grp, n in (("semantic_residual_vector_quantizer", min(nsem, nq)),
                       ("acoustic_residual_vector_quantizer", max(0, nq - nsem))):
            if n == 0:
                continue
            r = F.conv1d(emb, self.W[f"encoder.quantizer.{grp}.input_proj.weight"]).transpose(1, 2).double()
            for i in range(n):
                e = self.codebook(grp, i).double()
                d = ((r[:, :, None, :] - e[None, None]) ** 2).sum(-1)
                top = d.topk(2, -1, largest=False).values
                out.append((top[..., 1] - top[..., 0]) / top[..., 0].clamp(min=1e-30))
                r = r - e[d.argmin(-1)]
        return torch.stack(out, 1)

    def embeddings(self, wav: Tensor) -> Tensor:
        """wav [B, L] -> pre-quantizer embeddings [B, hidden, T12] (T:1230-1262)."""
        h = self.seanet(wav[:, None, :].float())
        h = self.transformer(h.transpose(1, 2)).transpose(1, 2)
        return mimi_conv(h, self.W["encoder.downsample.conv.weight"], None, stride=2, pad_mode="replicate")

    def encode(self, wavs: List) -> List[Tensor]:
        """Qwen3TTSTokenizer.encode (Z:208-257) -> V2Model.encode (K:960-990): right zero-pad the batch
        (EncodecFeatureExtractor padding), encode, keep valid_q codebooks and ceil(len / 1920) frames."""
        lens = [int(len(w)) for w in wavs]
        L = max(lens)
        x = torch.zeros(len(wavs), L)
        for i, w in enumerate(wavs):
            x[i, : lens[i]] = torch.as_tensor(w, dtype=torch.float32)
        codes = self.quantize(self.embeddings(x), self.valid_q)
        return [codes[i, :, : -(-n // self.down)].transpose(0, 1).contiguous() for i, n in enumerate(lens)]
