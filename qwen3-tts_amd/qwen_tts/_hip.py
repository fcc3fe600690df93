"""ctypes binding of libqwen3tts_amd.so (the C ABI declared in include/qwen3tts_amd.h).

The product path has no CPU fallback: `lib()` raises if the library or a GPU is missing.
Tensors are passed as raw device pointers (torch owns the memory; torch is plumbing here), the
stream as `torch.cuda.current_stream().cuda_stream`, so every launch is capturable into a HIP graph.
"""
from __future__ import annotations

import ctypes
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("QWEN3TTS_AMD_LIB",
                          os.path.join(os.path.dirname(HERE), "lib", "libqwen3tts_amd.so"))

F32, BF16 = 0, 1
ACT_NONE, ACT_SILU, ACT_GELU, ACT_RELU, ACT_SIGMOID, ACT_RELU_TANH = 0, 1, 2, 3, 4, 5
AACT_NONE, AACT_ELU = 0, 1
PAD_ZERO, PAD_REFLECT, PAD_REPLICATE = 0, 1, 2
EPI_STORE, EPI_ADD, EPI_SWIGLU = 0, 1, 2
ERRORS = {-1: "bad argument", -2: "bad shape", -3: "unsupported dtype", -4: "launch failed"}

c_int, c_ll, c_float, c_void_p, c_ull = ctypes.c_int, ctypes.c_longlong, ctypes.c_float, ctypes.c_void_p, ctypes.c_ulonglong


class GemmArgs(ctypes.Structure):
    _fields_ = [("M", c_int), ("N", c_int), ("K", c_int), ("a_dtype", c_int), ("w_dtype", c_int), ("o_dtype", c_int),
                ("A", c_void_p), ("lda", c_ll), ("a_index", c_void_p), ("W", c_void_p), ("gamma", c_void_p),
                ("eps", c_float), ("rmsnorm", c_int), ("bias", c_void_p), ("colscale", c_void_p), ("act", c_int), ("epi", c_int),
                ("out", c_void_p), ("ldo", c_ll), ("taps", c_int), ("dil", c_int), ("cin", c_int),
                ("cin_pad", c_int), ("t_in", c_int), ("t_out", c_int), ("t_off", c_int),
                ("ws", c_void_p), ("ws_bytes", c_ll), ("splitk", c_int),
                ("snake_alpha", c_void_p), ("snake_inv_beta", c_void_p), ("a_act", c_int),
                ("out2", c_void_p), ("ldo2", c_ll)]

GEMM_WS_MIN = 4 << 20  # QT_GEMM_WS_MIN


class QkvArgs(ctypes.Structure):
    _fields_ = [("R", c_int), ("Hq", c_int), ("Hkv", c_int), ("D", c_int), ("qkv", c_void_p), ("q_norm", c_void_p),
                ("k_norm", c_void_p), ("eps", c_float), ("cos_tab", c_void_p), ("sin_tab", c_void_p),
                ("rope_pos", c_void_p), ("row_batch", c_void_p), ("kv_pos", c_void_p), ("q_out", c_void_p),
                ("k_cache", c_void_p), ("v_cache", c_void_p), ("kv_dtype", c_int), ("Lmax", c_int)]


class AttnArgs(ctypes.Structure):
    _fields_ = [("R", c_int), ("Hq", c_int), ("Hkv", c_int), ("D", c_int), ("Lmax", c_int), ("window", c_int),
                ("q", c_void_p), ("k_cache", c_void_p), ("v_cache", c_void_p), ("kv_dtype", c_int),
                ("row_batch", c_void_p), ("row_start", c_void_p), ("row_len", c_void_p), ("out", c_void_p),
                ("o_dtype", c_int), ("max_keys", c_int)]


class DecodeAttnArgs(ctypes.Structure):
    _fields_ = [("R", c_int), ("Hq", c_int), ("Hkv", c_int), ("D", c_int), ("Lmax", c_int), ("window", c_int),
                ("qkv", c_void_p), ("q_norm", c_void_p), ("k_norm", c_void_p), ("eps", c_float),
                ("cos_tab", c_void_p), ("sin_tab", c_void_p), ("rope_pos", c_void_p), ("row_batch", c_void_p),
                ("kv_pos", c_void_p), ("row_start", c_void_p), ("k_cache", c_void_p), ("v_cache", c_void_p),
                ("kv_dtype", c_int), ("out", c_void_p), ("o_dtype", c_int), ("const_pos", c_int), ("nsplit", c_int),
                ("ws", c_void_p), ("ws_bytes", c_ll)]


class AttnOprojArgs(ctypes.Structure):
    _fields_ = [("R", c_int), ("Hq", c_int), ("Hkv", c_int), ("D", c_int), ("Lmax", c_int), ("qkv", c_void_p),
                ("q_norm", c_void_p), ("k_norm", c_void_p), ("eps", c_float), ("cos_tab", c_void_p), ("sin_tab", c_void_p),
                ("rope_pos", c_void_p), ("kv_pos", c_void_p), ("row_start", c_void_p), ("const_pos", c_int),
                ("k_cache", c_void_p), ("v_cache", c_void_p), ("kv_dtype", c_int), ("w_o", c_void_p), ("w_dtype", c_int),
                ("N", c_int), ("x", c_void_p), ("ldx", c_ll), ("x16", c_void_p), ("ldx16", c_ll), ("ws", c_void_p),
                ("ws_bytes", c_ll)]


P8 = c_void_p * 8


class CpStepArgs(ctypes.Structure):
    _fields_ = [("R", c_int), ("n_layers", c_int), ("Lmax", c_int), ("const_pos", c_int), ("V", c_int),
                ("eps", c_float), ("cos_tab", c_void_p), ("sin_tab", c_void_p),
                ("w_qkv", P8), ("w_o", P8), ("w_gu", P8), ("w_down", P8), ("q_norm", P8), ("k_norm", P8),
                ("k_cache", P8), ("v_cache", P8), ("w_lm", c_void_p), ("x", c_void_p), ("ldx", c_ll),
                ("qkv0", c_void_p), ("ldq", c_ll), ("logits", c_void_p), ("ldl", c_ll), ("ws", c_void_p),
                ("ws_bytes", c_ll)]


class TalkerStepArgs(ctypes.Structure):
    _fields_ = [("R", c_int), ("n_layers", c_int), ("Lmax", c_int), ("eps", ctypes.c_float), ("wtab", c_void_p),
                ("cos_tab", c_void_p), ("sin_tab", c_void_p), ("rope_pos", c_void_p), ("kv_pos", c_void_p),
                ("row_start", c_void_p), ("row_batch", c_void_p), ("x", c_void_p), ("ldx", c_ll), ("ws", c_void_p),
                ("ws_bytes", c_ll), ("first_layer", c_int), ("total_layers", c_int), ("qkv_in", c_void_p),
                ("ldq_in", c_ll), ("qkv_out", c_void_p), ("ldq_out", c_ll), ("att_in", c_void_p), ("lda_in", c_ll),
                ("att_out", c_void_p), ("lda_out", c_ll)]


class TalkerTailArgs(ctypes.Structure):
    _fields_ = [("R", c_int), ("eps", ctypes.c_float), ("att", c_void_p), ("lda", c_ll), ("x", c_void_p), ("ldx", c_ll),
                ("w_o", c_void_p), ("w_gu", c_void_p), ("w_down", c_void_p), ("w_qkv_next", c_void_p),
                ("qkv", c_void_p), ("ldq", c_ll), ("ws", c_void_p), ("ws_bytes", c_ll), ("H", c_int), ("I", c_int)]


class SampleArgs(ctypes.Structure):
    _fields_ = [("logits", c_void_p), ("R", c_int), ("V", c_int), ("ld", c_ll), ("seen", c_void_p),
                ("rep_penalty", c_float), ("n_generated", c_void_p), ("min_new_tokens", c_int), ("eos_id", c_int),
                ("suppress_lo", c_int), ("suppress_hi", c_int), ("suppress_keep", c_int), ("ignore_eos", c_int),
                ("finished", c_void_p), ("do_sample", c_int), ("top_k", c_int), ("top_p", c_float),
                ("temperature", c_float), ("seed", c_ull), ("step", c_void_p), ("substep", c_int),
                ("tok_out", c_void_p), ("codes", c_void_p), ("codes_ld", c_ll), ("codes_w", c_int),
                ("codes_col", c_int), ("codes_step_off", c_int), ("row_base", c_int),
                ("emb_table", c_void_p), ("emb_dim", c_int), ("emb_out", c_void_p), ("emb_ld", c_ll),
                ("seed_ptr", c_void_p), ("debug_u", c_float), ("emb_out16", c_void_p), ("emb_ld16", c_ll),
                ("emb2_table", c_void_p), ("emb2_dim", c_int), ("emb2_out", c_void_p), ("emb2_ld", c_ll),
                ("algo", c_int), ("ctr_stride", c_int), ("philox_row", c_void_p), ("force", c_void_p),
                ("pick", c_void_p)]


EXPORTS = ["qt_gemm", "qt_tile_weight", "qt_qkv_post", "qt_attention", "qt_decode_attention", "qt_decode_attn_ws_bytes",
           "qt_rmsnorm_rec", "qt_small_prefill_attention",
           "qt_decode_attn_oproj", "qt_attn_oproj_ws_bytes", "qt_attn_oproj_resident_blocks",
           "qt_cp_step", "qt_cp_prefill", "qt_cp_step_sampled", "qt_cp_step_ws_bytes", "qt_cp_step_supported", "qt_cp_step_dbg_bytes",
           "qt_talker_tail", "qt_talker_tail_ws_bytes", "qt_talker_tail_stamp_bytes", "qt_talker_tail_dbg_bytes",
           "qt_talker_tail_supported",
           "qt_sample", "qt_rmsnorm", "qt_gather_rows", "qt_frame_embed", "qt_advance", "qt_advance_rows",
           "qt_rvq_gather", "qt_snake", "qt_dwconv_ln", "qt_clamp_pcm",
           "qt_pad_time", "qt_zero_tail", "qt_layernorm", "qt_rvq_encode", "qt_rvq_encode_ws_bytes", "qt_mel_logmag", "qt_time_stats",
           "qt_scale_add", "qt_bcast_rows", "qt_build_id"]

_LIB = None
BUILD_ID = None  # qt_build_id() of the loaded library (digest of the sources it was built from)


def source_digest(probe=False):
    """Digest of the kernel sources shipped next to this package (qwen3-tts_amd/build.py's source_digest; the probe
    build's carries its flags and a "-probe" suffix), or None when they are absent (an installed copy without
    sources)."""
    bpath = os.path.join(os.path.dirname(HERE), "build.py")
    if not os.path.exists(bpath) or not os.path.isdir(os.path.join(os.path.dirname(HERE), "csrc")):
        return None
    import importlib.util
    spec = importlib.util.spec_from_file_location("_qt_build", bpath)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.source_digest(probe=probe) + ("-probe" if probe else "")


def load_library(path: str = LIB_PATH):
    """dlopen the library and declare signatures (no GPU needed; used by the CPU export test).  A library whose
    qt_build_id() differs from the digest of the kernel sources beside it is stale and refused (set
    QT_ALLOW_STALE_LIB=1 to load it anyway, e.g. for an A/B of an older build)."""
    if not os.path.exists(path):
        raise RuntimeError(f"HIP library not found at {path}: run `python qwen3-tts_amd/build.py` "
                           "(or __graft_entry__.build()); there is no CPU fallback")
    L = ctypes.CDLL(path)
    L.qt_build_id.restype = ctypes.c_char_p
    L.qt_build_id.argtypes = []
    bid = L.qt_build_id().decode()
    want = source_digest(probe=os.path.basename(path).endswith("_probe.so")) if path == LIB_PATH else None
    if want is not None and bid != want and os.environ.get("QT_ALLOW_STALE_LIB") != "1":
        raise RuntimeError(f"{path} was built from other sources (build id {bid}, sources {want}): rebuild with "
                           "`python qwen3-tts_amd/build.py`")
    global BUILD_ID
    BUILD_ID = bid
    P = c_void_p
    sig = {
        "qt_gemm": [P, P], "qt_tile_weight": [P, c_int, c_int, c_int, P, P], "qt_qkv_post": [P, P],
        "qt_attention": [P, P], "qt_decode_attention": [P, P], "qt_sample": [P, P],
        "qt_rmsnorm": [P, P, c_float, P, c_int, c_int, P],
        "qt_rmsnorm_rec": [P, P, c_float, P, c_int, c_int, P, c_ll, P, c_int, c_int, P],
        "qt_small_prefill_attention": [P, c_int, P],
        "qt_gather_rows": [P, c_int, P, c_int, c_int, P, c_ll, P],
        "qt_frame_embed": [P, P, c_int, c_int, c_int, c_int, c_int, P, c_ll, P, c_int, P, c_int, P, P, P, c_int, P],
        "qt_advance": [P, c_int, P],
        "qt_advance_rows": [P, c_int, c_int, c_int, P],
        "qt_rvq_gather": [P, c_int, c_int, c_int, c_int, P, c_int, c_int, P, P, P],
        "qt_snake": [P, P, c_int, c_ll, c_int, P, P, P],
        "qt_dwconv_ln": [P, c_int, c_int, c_int, c_int, P, P, P, P, c_float, P, P],
        "qt_clamp_pcm": [P, c_int, c_ll, P, P],
        "qt_decode_attn_ws_bytes": [c_int, c_int, c_int, c_int, c_int],
        "qt_decode_attn_oproj": [P, P],
        "qt_attn_oproj_ws_bytes": [c_int, c_int],
        "qt_attn_oproj_resident_blocks": [],
        "qt_cp_step": [P, P], "qt_cp_prefill": [P, P], "qt_cp_step_sampled": [P, P, P], "qt_cp_step_ws_bytes": [], "qt_cp_step_dbg_bytes": [],
        "qt_cp_step_supported": [c_int, c_int, c_int, c_int, c_int, c_int, c_int],
        "qt_talker_tail": [P, P], "qt_talker_tail_ws_bytes": [], "qt_talker_tail_stamp_bytes": [], "qt_talker_tail_dbg_bytes": [],
        "qt_talker_tail_supported": [c_int, c_int, c_int, c_int, c_int],
        "qt_pad_time": [P, c_ll, P, c_ll, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, P, c_ll, P],
        "qt_zero_tail": [P, c_int, c_int, c_int, c_int, c_int, c_ll, P],
        "qt_layernorm": [P, c_ll, P, P, c_float, P, c_int, c_ll, c_int, c_int, P],
        "qt_rvq_encode": [P, c_ll, P, P, c_int, c_int, c_int, c_int, P, c_ll, P, c_ll, P],
        "qt_rvq_encode_ws_bytes": [c_int, c_int, c_int],
        "qt_mel_logmag": [P, c_ll, c_int, c_int, P, c_int, P, c_ll, P],
        "qt_time_stats": [P, c_int, c_ll, P, c_ll, c_int, c_int, c_int, c_float, P, P, c_ll, P],
        "qt_scale_add": [P, c_ll, P, c_ll, P, c_ll, c_int, c_int, c_int, c_int, P, c_ll, P],
        "qt_bcast_rows": [P, c_ll, c_int, c_int, c_int, P, c_int, c_ll, P],
    }
    for name, args in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = c_ll if name.endswith("_ws_bytes") else c_int
    return L


def lib():
    global _LIB
    if _LIB is None:
        if not torch.cuda.is_available():
            raise RuntimeError("qwen_tts (MI355X build) needs a ROCm GPU: no device visible and no CPU fallback")
        _LIB = load_library()
    return _LIB


def env_int(name: str, default: int) -> int:
    """An integer environment knob parsed like C atoi (as the library's own getenv knobs are): optional leading
    whitespace and sign, then digits; anything else (empty, 'off') is 0.  Unset -> default."""
    v = os.environ.get(name)
    if v is None:
        return default
    import re
    m = re.match(r"\s*([+-]?\d+)", v)
    return int(m.group(1)) if m else 0


# the probe library (build.py --probe) reads the measurement knobs; the product library ignores the environment, and
# so do the host-side mirrors of its knobs (lib_knob)
PROBE = os.path.basename(LIB_PATH).endswith("_probe.so")


def lib_knob(name: str, default: int) -> int:
    """A knob the library reads too (e.g. QT_PF): honoured only with the probe library, like the library's own."""
    return env_int(name, default) if PROBE else default


def check(rc: int, what: str):
    if rc != 0:
        raise RuntimeError(f"{what} failed: {ERRORS.get(rc, rc)}")


def ptr(t):
    return None if t is None else t.data_ptr()


def stream():
    return torch.cuda.current_stream().cuda_stream


def dtype_code(dt: torch.dtype) -> int:
    if dt == torch.float32:
        return F32
    if dt == torch.bfloat16:
        return BF16
    raise ValueError(f"unsupported dtype {dt}")
