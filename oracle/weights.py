"""Seeded synthetic weights for the oracle and the golden fixtures.

TEST INFRASTRUCTURE (oracle/): only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this package.  The product path never does.

No checkpoint exists in this container or on the GPU box, so every parity run uses
seeded synthetic weights.  Each parameter is drawn from its own numpy PCG64 stream keyed by
(seed, crc32(parameter name)), so the same name/shape always gets the same values whichever process
asks, in whatever order.  Parameter names are the reference checkpoint keys (state_dict names of
`Qwen3TTSForConditionalGeneration` / `Qwen3TTSTokenizerV2Model`), so a dict from here is exactly what a
real `model.safetensors` would hold.
"""
from __future__ import annotations

import re
import zlib

import numpy as np

_TRANSPOSED_CONV = re.compile(r"(decoder\.upsample\.\d+\.0\.conv|decoder\.decoder\.\d+\.block\.1\.conv)\.weight$")


_FINAL_CONV = re.compile(r"decoder\.decoder\.\d+\.conv\.weight$")


def _rng(seed: int, name: str) -> np.random.Generator:
    return np.random.default_rng([int(seed), zlib.crc32(name.encode())])


def synth_param(name: str, shape, seed: int = 1234) -> np.ndarray:
    """Deterministic float32 value for one parameter (sigma rules: SURVEY.md §8c, fan-in scaled convs)."""
    shape = tuple(int(s) for s in shape)
    g = _rng(seed, name)
    n = lambda: g.standard_normal(shape, dtype=np.float32)  # noqa: E731
    if name.endswith("_codebook.cluster_usage") or name.endswith(".codebook.cluster_usage"):
        return g.uniform(0.5, 2.0, shape).astype(np.float32)
    if name.endswith("_codebook.embedding_sum") or name.endswith(".codebook.embed_sum"):
        return n()
    if name.endswith(".codebook.initialized"):
        return np.ones(shape, np.float32)
    if (name.startswith("encoder.") or name.startswith("speaker_encoder.")) and name.endswith("weight") \
            and len(shape) in (2, 3) and "norm" not in name:
        # tokenizer encoder (Mimi) / ECAPA convs and linears: fan-in scaled so activations stay O(1)
        fan_in = shape[1] * (shape[2] if len(shape) == 3 else 1)
        gain = 1.0
        if name.startswith("speaker_encoder."):
            gain = 1.4  # ReLU
        elif name.endswith("block.3.conv.weight"):
            gain = 0.5  # resnet-block output onto the residual stream
        return (gain * n() / np.sqrt(fan_in)).astype(np.float32)
    if name.endswith(".alpha") or name.endswith(".beta"):  # SnakeBeta (log-scale params)
        return (0.1 * n()).astype(np.float32)
    if name.endswith("layer_scale.scale") or name.endswith(".gamma"):
        return (0.1 + 0.01 * n()).astype(np.float32)
    if name.endswith("norm.weight") or name.endswith("layernorm.weight"):
        return (1.0 + 0.1 * n()).astype(np.float32)
    if name.endswith(".bias"):
        return (0.02 * n()).astype(np.float32)
    if name.startswith("decoder.") and len(shape) in (2, 3):  # codec convs / linears: fan-in scaled
        if len(shape) == 2:
            fan_in = shape[1]
        elif _TRANSPOSED_CONV.search(name):
            fan_in = shape[0] * 2
        else:
            fan_in = shape[1] * shape[2]
        gain = 1.0
        if name.endswith("conv2.conv.weight"):  # residual-unit output: keep the residual stream O(1)
            gain = 0.25
        elif _FINAL_CONV.search(name):          # waveform head: PCM well inside the clamp(-1, 1)
            gain = 0.35
        return (gain * n() / np.sqrt(fan_in)).astype(np.float32)
    return (0.02 * n()).astype(np.float32)


def synth_state_dict(specs, seed: int = 1234, threads: int = 0):
    """specs: iterable of (name, shape) -> {name: np.float32 array}.  threads > 0 draws the parameters on a thread
    pool (each has its own generator, so the values do not depend on the order or the pool size)."""
    specs = list(specs)
    if threads > 0:
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(threads) as ex:
            vals = list(ex.map(lambda ns: synth_param(ns[0], ns[1], seed), specs))
        return {name: v for (name, _), v in zip(specs, vals)}
    return {name: synth_param(name, shape, seed) for name, shape in specs}
