"""CPU fp32 restatement of the Qwen3-TTS-Tokenizer-12Hz codec decoder.

TEST INFRASTRUCTURE (oracle/): parity checker for the HIP codec path; never imported by the product.

`K` = qwen_tts/core/tokenizer_12hz/modeling_qwen3_tts_tokenizer_v2.py, `Z` = qwen_tts/inference/qwen3_tts_tokenizer.py.
Layout here is the reference's channels-first [B, C, T].
"""
from __future__ import annotations

import math
from typing import Dict, List

import torch
import torch.nn.functional as F

from .talker import rmsnorm, rope_cos_sin, apply_rope

Tensor = torch.Tensor


def codec_param_specs(ccfg: dict):
    """(name, shape) of every decoder parameter (K:823-866 and the modules it builds)."""
    d = ccfg["decoder_config"]
    cd, lat, hid, ds = d["codebook_dim"], d["latent_dim"], d["hidden_size"], d["decoder_dim"]
    heads = d["num_attention_heads"]
    hd = hid // heads
    nkv = d["num_key_value_heads"]
    specs = []
    half = cd // 2
    specs += [("decoder.quantizer.rvq_first.output_proj.weight", (cd, half, 1)),
              ("decoder.quantizer.rvq_rest.output_proj.weight", (cd, half, 1)),
              # encode-side projections (K:757-759): present in checkpoints, unused by decode
              ("decoder.quantizer.rvq_first.input_proj.weight", (half, cd, 1)),
              ("decoder.quantizer.rvq_rest.input_proj.weight", (half, cd, 1))]
    for grp, n in (("rvq_first", 1), ("rvq_rest", d["num_quantizers"] - 1)):
        for i in range(n):
            p = f"decoder.quantizer.{grp}.vq.layers.{i}._codebook"
            specs += [(f"{p}.cluster_usage", (d["codebook_size"],)), (f"{p}.embedding_sum", (d["codebook_size"], half))]
    specs += [("decoder.pre_conv.conv.weight", (lat, cd, 3)), ("decoder.pre_conv.conv.bias", (lat,))]
    pt = "decoder.pre_transformer"
    specs += [(f"{pt}.input_proj.weight", (hid, lat)), (f"{pt}.input_proj.bias", (hid,)),
              (f"{pt}.output_proj.weight", (lat, hid)), (f"{pt}.output_proj.bias", (lat,)),
              (f"{pt}.norm.weight", (hid,))]
    for i in range(d["num_hidden_layers"]):
        p = f"{pt}.layers.{i}"
        specs += [(f"{p}.self_attn.q_proj.weight", (heads * hd, hid)), (f"{p}.self_attn.k_proj.weight", (nkv * hd, hid)),
                  (f"{p}.self_attn.v_proj.weight", (nkv * hd, hid)), (f"{p}.self_attn.o_proj.weight", (hid, heads * hd)),
                  (f"{p}.mlp.gate_proj.weight", (d["intermediate_size"], hid)),
                  (f"{p}.mlp.up_proj.weight", (d["intermediate_size"], hid)),
                  (f"{p}.mlp.down_proj.weight", (hid, d["intermediate_size"])),
                  (f"{p}.input_layernorm.weight", (hid,)), (f"{p}.post_attention_layernorm.weight", (hid,)),
                  (f"{p}.self_attn_layer_scale.scale", (hid,)), (f"{p}.mlp_layer_scale.scale", (hid,))]
    for i, f in enumerate(d["upsampling_ratios"]):
        p = f"decoder.upsample.{i}"
        specs += [(f"{p}.0.conv.weight", (lat, lat, f)), (f"{p}.0.conv.bias", (lat,)),
                  (f"{p}.1.dwconv.conv.weight", (lat, 1, 7)), (f"{p}.1.dwconv.conv.bias", (lat,)),
                  (f"{p}.1.norm.weight", (lat,)), (f"{p}.1.norm.bias", (lat,)),
                  (f"{p}.1.pwconv1.weight", (4 * lat, lat)), (f"{p}.1.pwconv1.bias", (4 * lat,)),
                  (f"{p}.1.pwconv2.weight", (lat, 4 * lat)), (f"{p}.1.pwconv2.bias", (lat,)),
                  (f"{p}.1.gamma", (lat,))]
    specs += [("decoder.decoder.0.conv.weight", (ds, lat, 7)), ("decoder.decoder.0.conv.bias", (ds,))]
    for i, r in enumerate(d["upsample_rates"]):
        cin, cout = ds // 2 ** i, ds // 2 ** (i + 1)
        p = f"decoder.decoder.{i + 1}.block"
        specs += [(f"{p}.0.alpha", (cin,)), (f"{p}.0.beta", (cin,)),
                  (f"{p}.1.conv.weight", (cin, cout, 2 * r)), (f"{p}.1.conv.bias", (cout,))]
        for j in range(3):
            q = f"{p}.{j + 2}"
            specs += [(f"{q}.act1.alpha", (cout,)), (f"{q}.act1.beta", (cout,)),
                      (f"{q}.conv1.conv.weight", (cout, cout, 7)), (f"{q}.conv1.conv.bias", (cout,)),
                      (f"{q}.act2.alpha", (cout,)), (f"{q}.act2.beta", (cout,)),
                      (f"{q}.conv2.conv.weight", (cout, cout, 1)), (f"{q}.conv2.conv.bias", (cout,))]
    n = len(d["upsample_rates"])
    cl = ds // 2 ** n
    specs += [(f"decoder.decoder.{n + 1}.alpha", (cl,)), (f"decoder.decoder.{n + 1}.beta", (cl,)),
              (f"decoder.decoder.{n + 2}.conv.weight", (1, cl, 7)), (f"decoder.decoder.{n + 2}.conv.bias", (1,))]
    return specs


def causal_conv(x, w, b, dilation=1, groups=1):
    """Qwen3TTSTokenizerV2CausalConvNet (K:159-192): left pad (k-1)*d, extra right pad 0 at stride 1."""
    k = (w.shape[-1] - 1) * dilation + 1
    return F.conv1d(F.pad(x, (k - 1, 0)), w, b, dilation=dilation, groups=groups)


def trans_conv(x, w, b, stride):
    """Qwen3TTSTokenizerV2CausalTransConvNet (K:195-207): ConvTranspose1d then trim (k - s) each side."""
    y = F.conv_transpose1d(x, w, b, stride=stride)
    pad = w.shape[-1] - stride
    return y[..., pad: y.shape[-1] - pad]


def snake(x, alpha, beta):
    """SnakeBeta (K:577-615): x + 1/(exp(beta)+1e-9) * sin(x*exp(alpha))^2."""
    a = torch.exp(alpha)[None, :, None]
    bb = torch.exp(beta)[None, :, None]
    return x + (1.0 / (bb + 1e-9)) * torch.pow(torch.sin(x * a), 2)


class CodecOracle:
    def __init__(self, ccfg: dict, weights: Dict[str, Tensor]):
        self.ccfg = ccfg
        self.d = ccfg["decoder_config"]
        self.W = {k: (v if isinstance(v, Tensor) else torch.from_numpy(v)).float() for k, v in weights.items()}

    # C1
    def dequant(self, codes):
        """SplitResidualVectorQuantizer.decode (K:814-820, 772-776, 706-710, 675-678). codes [B,16,T]."""
        W = self.W
        out = None
        for grp, idx in (("rvq_first", range(0, 1)), ("rvq_rest", range(1, self.d["num_quantizers"]))):
            q = None
            for j, i in enumerate(idx):
                p = f"decoder.quantizer.{grp}.vq.layers.{j}._codebook"
                table = W[f"{p}.embedding_sum"] / W[f"{p}.cluster_usage"].clamp(min=1e-5)[:, None]
                e = F.embedding(codes[:, i], table).transpose(1, 2)
                q = e if q is None else q + e
            q = F.conv1d(q, W[f"decoder.quantizer.{grp}.output_proj.weight"])
            out = q if out is None else out + q
        return out

    # C3
    def transformer(self, x):
        """Qwen3TTSTokenizerV2DecoderTransformerModel.forward (K:500-574), x [B,T,lat]."""
        d, W = self.d, self.W
        pt = "decoder.pre_transformer"
        x = x @ W[f"{pt}.input_proj.weight"].T + W[f"{pt}.input_proj.bias"]
        B, T, hid = x.shape
        heads = d["num_attention_heads"]
        hd = hid // heads
        pos = torch.arange(T)
        cos, sin = rope_cos_sin(pos[None].expand(B, T), hd, d["rope_theta"])
        kv = torch.arange(T)
        allowed = (kv[None, :] <= pos[:, None]) & (kv[None, :] > pos[:, None] - d["sliding_window"])
        add = torch.zeros(T, T).masked_fill(~allowed, torch.finfo(torch.float32).min)[None, None]
        eps = d["rms_norm_eps"]
        for i in range(d["num_hidden_layers"]):
            p = f"{pt}.layers.{i}"
            h = rmsnorm(x, W[f"{p}.input_layernorm.weight"], eps)
            q = (h @ W[f"{p}.self_attn.q_proj.weight"].T).view(B, T, heads, hd).transpose(1, 2)
            k = (h @ W[f"{p}.self_attn.k_proj.weight"].T).view(B, T, -1, hd).transpose(1, 2)
            v = (h @ W[f"{p}.self_attn.v_proj.weight"].T).view(B, T, -1, hd).transpose(1, 2)
            q, k = apply_rope(q, cos, sin), apply_rope(k, cos, sin)
            rep = heads // k.shape[1]
            if rep > 1:
                k, v = k.repeat_interleave(rep, 1), v.repeat_interleave(rep, 1)
            s = torch.matmul(q, k.transpose(2, 3)) * hd ** -0.5 + add
            a = torch.matmul(torch.softmax(s, -1, dtype=torch.float32), v).transpose(1, 2).reshape(B, T, hid)
            x = x + W[f"{p}.self_attn_layer_scale.scale"] * (a @ W[f"{p}.self_attn.o_proj.weight"].T)
            h = rmsnorm(x, W[f"{p}.post_attention_layernorm.weight"], eps)
            m = F.silu(h @ W[f"{p}.mlp.gate_proj.weight"].T) * (h @ W[f"{p}.mlp.up_proj.weight"].T)
            x = x + W[f"{p}.mlp_layer_scale.scale"] * (m @ W[f"{p}.mlp.down_proj.weight"].T)
        x = rmsnorm(x, W[f"{pt}.norm.weight"], eps)
        return x @ W[f"{pt}.output_proj.weight"].T + W[f"{pt}.output_proj.bias"]

    def convnext(self, x, p):
        """Qwen3TTSTokenizerV2ConvNeXtBlock (K:210-242)."""
        W = self.W
        h = causal_conv(x, W[f"{p}.dwconv.conv.weight"], W[f"{p}.dwconv.conv.bias"], groups=x.shape[1])
        h = F.layer_norm(h.permute(0, 2, 1), (x.shape[1],), W[f"{p}.norm.weight"], W[f"{p}.norm.bias"], 1e-6)
        h = F.gelu(h @ W[f"{p}.pwconv1.weight"].T + W[f"{p}.pwconv1.bias"])
        h = h @ W[f"{p}.pwconv2.weight"].T + W[f"{p}.pwconv2.bias"]
        return x + (W[f"{p}.gamma"] * h).permute(0, 2, 1)

    def forward(self, codes):
        """Qwen3TTSTokenizerV2Decoder.forward (K:868-883). codes [B,16,T] -> wav [B,1,1920T-555]."""
        d, W = self.d, self.W
        h = self.dequant(codes)
        h = causal_conv(h, W["decoder.pre_conv.conv.weight"], W["decoder.pre_conv.conv.bias"]).transpose(1, 2)
        h = self.transformer(h).permute(0, 2, 1)
        for i, f in enumerate(d["upsampling_ratios"]):
            h = trans_conv(h, W[f"decoder.upsample.{i}.0.conv.weight"], W[f"decoder.upsample.{i}.0.conv.bias"], f)
            h = self.convnext(h, f"decoder.upsample.{i}.1")
        h = causal_conv(h, W["decoder.decoder.0.conv.weight"], W["decoder.decoder.0.conv.bias"])
        for i, r in enumerate(d["upsample_rates"]):
            p = f"decoder.decoder.{i + 1}.block"
            h = snake(h, W[f"{p}.0.alpha"], W[f"{p}.0.beta"])
            h = trans_conv(h, W[f"{p}.1.conv.weight"], W[f"{p}.1.conv.bias"], r)
            for j, dil in enumerate((1, 3, 9)):
                q = f"{p}.{j + 2}"
                res = h
                h = snake(h, W[f"{q}.act1.alpha"], W[f"{q}.act1.beta"])
                h = causal_conv(h, W[f"{q}.conv1.conv.weight"], W[f"{q}.conv1.conv.bias"], dilation=dil)
                h = snake(h, W[f"{q}.act2.alpha"], W[f"{q}.act2.beta"])
                h = causal_conv(h, W[f"{q}.conv2.conv.weight"], W[f"{q}.conv2.conv.bias"]) + res
        n = len(d["upsample_rates"])
        h = snake(h, W[f"decoder.decoder.{n + 1}.alpha"], W[f"decoder.decoder.{n + 1}.beta"])
        h = causal_conv(h, W[f"decoder.decoder.{n + 2}.conv.weight"], W[f"decoder.decoder.{n + 2}.conv.bias"])
        return h.clamp(-1, 1)

    def total_upsample(self):
        return int(math.prod(self.d["upsample_rates"]) * math.prod(self.d["upsampling_ratios"]))

    def chunked_decode(self, codes, chunk_size=300, left_context_size=25):
        """Qwen3TTSTokenizerV2Decoder.chunked_decode (K:885-895)."""
        wavs, start, up = [], 0, self.total_upsample()
        while start < codes.shape[-1]:
            end = min(start + chunk_size, codes.shape[-1])
            ctx = left_context_size if start - left_context_size > 0 else start
            w = self.forward(codes[..., start - ctx:end])
            wavs.append(w[..., ctx * up:])
            start = end
        return torch.cat(wavs, -1)

    def decode(self, audio_codes: Tensor) -> List[Tensor]:
        """Qwen3TTSTokenizerV2Model.decode (K:992-1022): audio_codes [B,T,16] -> list of 1-D wavs."""
        wav = self.chunked_decode(audio_codes.transpose(1, 2)).squeeze(1)
        lengths = (audio_codes[..., 0] > 0).sum(1) * self.ccfg["decode_upsample_rate"]
        return [a[:l] for a, l in zip(wav, lengths)]


def tokenizer_decode(o: CodecOracle, codes_list):
    """Qwen3TTSTokenizer.decode list path (Z:259-365): right-pad with code 0, decode, numpy float32."""
    codes = [torch.as_tensor(c, dtype=torch.long) for c in codes_list]
    padded = torch.nn.utils.rnn.pad_sequence(codes, batch_first=True, padding_value=0)
    return [w.float().numpy() for w in o.decode(padded)]
