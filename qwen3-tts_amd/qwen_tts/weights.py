"""Checkpoint loading for the MI355X engine.

Sources, in order: `model.safetensors` (+ sharded `model-*.safetensors`) in the checkpoint directory,
keyed by the reference's state_dict names; otherwise seeded synthetic weights
generated directly on the GPU (no checkpoint exists offline).  Synthetic weights follow the same sigma
rules as the parity fixtures but use torch's device RNG: they are for benchmarking, not parity.
"""
from __future__ import annotations

import glob
import json
import os
import re
import warnings
from typing import Dict

import torch

PRESETS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "configs")
HUB_ALIASES = {
    "qwen/qwen3-tts-12hz-1.7b-customvoice": "1.7b-customvoice",
    "qwen/qwen3-tts-12hz-1.7b-voicedesign": "1.7b-voicedesign",
    "qwen/qwen3-tts-12hz-1.7b-base": "1.7b-base",
    "qwen/qwen3-tts-12hz-0.6b-customvoice": "0.6b-customvoice",
    "qwen/qwen3-tts-12hz-0.6b-base": "0.6b-base",
    "qwen/qwen3-tts-tokenizer-12hz": "1.7b-customvoice/speech_tokenizer",
}


def resolve_path(name_or_path: str) -> str:
    """Local checkpoint dir, a packaged synthetic preset name, or a hub id mapped to its preset."""
    if os.path.isdir(name_or_path):
        return name_or_path
    key = name_or_path.rstrip("/").lower()
    if key.startswith("synthetic:"):
        key = key.split(":", 1)[1]
    key = HUB_ALIASES.get(key, key)
    p = os.path.join(PRESETS, key)
    if os.path.isdir(p):
        if not name_or_path.lower().startswith("synthetic:"):
            warnings.warn(f"{name_or_path!r} is not available offline: using the synthetic-weight preset {key!r} "
                          "(real dims where known, ASSUMED elsewhere; see SURVEY.md §8.0)")
        return p
    raise FileNotFoundError(f"no checkpoint directory or preset for {name_or_path!r}")


def is_preset_dir(d: str) -> bool:
    """True for the packaged synthetic-weight presets (the only directories allowed to have no weights)."""
    return os.path.abspath(d).startswith(os.path.abspath(PRESETS) + os.sep)


def read_json(path):
    with open(path) as f:
        return json.load(f)


def load_safetensors(d: str) -> Dict[str, torch.Tensor]:
    files = sorted(glob.glob(os.path.join(d, "model*.safetensors")))
    if not files:
        return {}
    from safetensors.torch import load_file
    out = {}
    for f in files:
        out.update(load_file(f))
    return out


_TRANSPOSED = re.compile(r"(decoder\.upsample\.\d+\.0\.conv|decoder\.decoder\.\d+\.block\.1\.conv)\.weight$")


def synthetic(specs, device, seed=1234) -> Dict[str, torch.Tensor]:
    """Seeded synthetic weights on the device (benchmark use)."""
    g = torch.Generator(device=device).manual_seed(seed)
    out = {}
    for name, shape in specs:
        n = lambda: torch.randn(shape, generator=g, device=device)  # noqa: E731
        if name.endswith("_codebook.cluster_usage") or name.endswith(".codebook.cluster_usage"):
            t = torch.rand(shape, generator=g, device=device) * 1.5 + 0.5
        elif name.endswith("_codebook.embedding_sum") or name.endswith(".codebook.embed_sum"):
            t = n()
        elif name.endswith(".codebook.initialized"):
            t = torch.ones(shape, device=device)
        elif (name.startswith("encoder.") or name.startswith("speaker_encoder.")) and name.endswith("weight") \
                and len(shape) in (2, 3) and "norm" not in name:
            fan = shape[1] * (shape[2] if len(shape) == 3 else 1)
            gain = 1.4 if name.startswith("speaker_encoder.") else (0.5 if name.endswith("block.3.conv.weight") else 1.0)
            t = gain * n() / fan ** 0.5
        elif name.endswith(".alpha") or name.endswith(".beta"):
            t = 0.1 * n()
        elif name.endswith("layer_scale.scale") or name.endswith(".gamma"):
            t = 0.1 + 0.01 * n()
        elif name.endswith("norm.weight"):
            t = 1.0 + 0.1 * n()
        elif name.endswith(".bias"):
            t = 0.02 * n()
        elif name.startswith("decoder.") and len(shape) in (2, 3):
            fan = shape[1] if len(shape) == 2 else (shape[0] * 2 if _TRANSPOSED.search(name) else shape[1] * shape[2])
            gain = 0.25 if name.endswith("conv2.conv.weight") else 1.0
            t = gain * n() / fan ** 0.5
        else:
            t = 0.02 * n()
        out[name] = t
    return out


def _layer_specs(prefix, hidden, inter, heads, kv, hd):
    return [(f"{prefix}.self_attn.q_proj.weight", (heads * hd, hidden)), (f"{prefix}.self_attn.k_proj.weight", (kv * hd, hidden)),
            (f"{prefix}.self_attn.v_proj.weight", (kv * hd, hidden)), (f"{prefix}.self_attn.o_proj.weight", (hidden, heads * hd)),
            (f"{prefix}.self_attn.q_norm.weight", (hd,)), (f"{prefix}.self_attn.k_norm.weight", (hd,)),
            (f"{prefix}.mlp.gate_proj.weight", (inter, hidden)), (f"{prefix}.mlp.up_proj.weight", (inter, hidden)),
            (f"{prefix}.mlp.down_proj.weight", (hidden, inter)), (f"{prefix}.input_layernorm.weight", (hidden,)),
            (f"{prefix}.post_attention_layernorm.weight", (hidden,))]


def talker_specs(cfg):
    """Names/shapes of the talker + code predictor parameters (reference state_dict keys)."""
    t = cfg["talker_config"]
    c = t["code_predictor_config"]
    H, thd, G = t["hidden_size"], t["text_hidden_size"], t["num_code_groups"]
    s = []
    for i in range(t["num_hidden_layers"]):
        s += _layer_specs(f"talker.model.layers.{i}", H, t["intermediate_size"], t["num_attention_heads"],
                          t["num_key_value_heads"], t["head_dim"])
    s += [("talker.model.norm.weight", (H,)), ("talker.model.codec_embedding.weight", (t["vocab_size"], H)),
          ("talker.model.text_embedding.weight", (t["text_vocab_size"], thd)),
          ("talker.text_projection.linear_fc1.weight", (thd, thd)), ("talker.text_projection.linear_fc1.bias", (thd,)),
          ("talker.text_projection.linear_fc2.weight", (H, thd)), ("talker.text_projection.linear_fc2.bias", (H,)),
          ("talker.codec_head.weight", (t["vocab_size"], H))]
    Hc = c["hidden_size"]
    for i in range(c["num_hidden_layers"]):
        s += _layer_specs(f"talker.code_predictor.model.layers.{i}", Hc, c["intermediate_size"],
                          c["num_attention_heads"], c["num_key_value_heads"], c["head_dim"])
    s.append(("talker.code_predictor.model.norm.weight", (Hc,)))
    s += [(f"talker.code_predictor.model.codec_embedding.{g}.weight", (c["vocab_size"], H)) for g in range(G - 1)]
    s += [(f"talker.code_predictor.lm_head.{g}.weight", (c["vocab_size"], Hc)) for g in range(G - 1)]
    if Hc != H:
        s += [("talker.code_predictor.small_to_mtp_projection.weight", (Hc, H)),
              ("talker.code_predictor.small_to_mtp_projection.bias", (Hc,))]
    return s


def codec_specs(ccfg):
    """Names/shapes of the 12 Hz decoder parameters used by decode."""
    d = ccfg["decoder_config"]
    cd, lat, hid, ds = d["codebook_dim"], d["latent_dim"], d["hidden_size"], d["decoder_dim"]
    heads, nkv, I = d["num_attention_heads"], d["num_key_value_heads"], d["intermediate_size"]
    hd, half = hid // heads, cd // 2
    s = [("decoder.quantizer.rvq_first.output_proj.weight", (cd, half, 1)),
         ("decoder.quantizer.rvq_rest.output_proj.weight", (cd, half, 1))]
    for grp, n in (("rvq_first", 1), ("rvq_rest", d["num_quantizers"] - 1)):
        for i in range(n):
            p = f"decoder.quantizer.{grp}.vq.layers.{i}._codebook"
            s += [(f"{p}.cluster_usage", (d["codebook_size"],)), (f"{p}.embedding_sum", (d["codebook_size"], half))]
    pt = "decoder.pre_transformer"
    s += [("decoder.pre_conv.conv.weight", (lat, cd, 3)), ("decoder.pre_conv.conv.bias", (lat,)),
          (f"{pt}.input_proj.weight", (hid, lat)), (f"{pt}.input_proj.bias", (hid,)),
          (f"{pt}.output_proj.weight", (lat, hid)), (f"{pt}.output_proj.bias", (lat,)), (f"{pt}.norm.weight", (hid,))]
    for i in range(d["num_hidden_layers"]):
        p = f"{pt}.layers.{i}"
        s += [(f"{p}.self_attn.q_proj.weight", (heads * hd, hid)), (f"{p}.self_attn.k_proj.weight", (nkv * hd, hid)),
              (f"{p}.self_attn.v_proj.weight", (nkv * hd, hid)), (f"{p}.self_attn.o_proj.weight", (hid, heads * hd)),
              (f"{p}.mlp.gate_proj.weight", (I, hid)), (f"{p}.mlp.up_proj.weight", (I, hid)),
              (f"{p}.mlp.down_proj.weight", (hid, I)), (f"{p}.input_layernorm.weight", (hid,)),
              (f"{p}.post_attention_layernorm.weight", (hid,)), (f"{p}.self_attn_layer_scale.scale", (hid,)),
              (f"{p}.mlp_layer_scale.scale", (hid,))]
    for i, f in enumerate(d["upsampling_ratios"]):
        p = f"decoder.upsample.{i}"
        s += [(f"{p}.0.conv.weight", (lat, lat, f)), (f"{p}.0.conv.bias", (lat,)), (f"{p}.1.dwconv.conv.weight", (lat, 1, 7)),
              (f"{p}.1.dwconv.conv.bias", (lat,)), (f"{p}.1.norm.weight", (lat,)), (f"{p}.1.norm.bias", (lat,)),
              (f"{p}.1.pwconv1.weight", (4 * lat, lat)), (f"{p}.1.pwconv1.bias", (4 * lat,)),
              (f"{p}.1.pwconv2.weight", (lat, 4 * lat)), (f"{p}.1.pwconv2.bias", (lat,)), (f"{p}.1.gamma", (lat,))]
    s += [("decoder.decoder.0.conv.weight", (ds, lat, 7)), ("decoder.decoder.0.conv.bias", (ds,))]
    for i, r in enumerate(d["upsample_rates"]):
        cin, cout = ds // 2 ** i, ds // 2 ** (i + 1)
        p = f"decoder.decoder.{i + 1}.block"
        s += [(f"{p}.0.alpha", (cin,)), (f"{p}.0.beta", (cin,)), (f"{p}.1.conv.weight", (cin, cout, 2 * r)),
              (f"{p}.1.conv.bias", (cout,))]
        for j in range(3):
            q = f"{p}.{j + 2}"
            s += [(f"{q}.act1.alpha", (cout,)), (f"{q}.act1.beta", (cout,)), (f"{q}.conv1.conv.weight", (cout, cout, 7)),
                  (f"{q}.conv1.conv.bias", (cout,)), (f"{q}.act2.alpha", (cout,)), (f"{q}.act2.beta", (cout,)),
                  (f"{q}.conv2.conv.weight", (cout, cout, 1)), (f"{q}.conv2.conv.bias", (cout,))]
    n = len(d["upsample_rates"])
    cl = ds // 2 ** n
    s += [(f"decoder.decoder.{n + 1}.alpha", (cl,)), (f"decoder.decoder.{n + 1}.beta", (cl,)),
          (f"decoder.decoder.{n + 2}.conv.weight", (1, cl, 7)), (f"decoder.decoder.{n + 2}.conv.bias", (1,))]
    return s
