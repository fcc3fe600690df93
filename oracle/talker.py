"""CPU fp32 restatement of the Qwen3-TTS AR decoder: talker backbone, code predictor, prompt
assembly and the HF-4.57 generation loop.

TEST INFRASTRUCTURE (oracle/): the parity checker for the HIP path.  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may import it; the product never does.

Every function cites the reference lines it restates (paths relative to /root/reference,
`M` = qwen_tts/core/models/modeling_qwen3_tts.py).  Weights are a dict keyed by the reference
checkpoint names (see oracle/weights.py).  Pinned against golden vectors produced by the reference
itself (tests/golden/make_golden.py, tests/test_oracle_golden.py).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import torch
import torch.nn.functional as F

Tensor = torch.Tensor


# ----------------------------------------------------------------------------------------------
# parameter inventory (names/shapes == reference state_dict keys)
# ----------------------------------------------------------------------------------------------

def _layer_specs(prefix, hidden, inter, heads, kv, hd):
    return [
        (f"{prefix}.self_attn.q_proj.weight", (heads * hd, hidden)),
        (f"{prefix}.self_attn.k_proj.weight", (kv * hd, hidden)),
        (f"{prefix}.self_attn.v_proj.weight", (kv * hd, hidden)),
        (f"{prefix}.self_attn.o_proj.weight", (hidden, heads * hd)),
        (f"{prefix}.self_attn.q_norm.weight", (hd,)),
        (f"{prefix}.self_attn.k_norm.weight", (hd,)),
        (f"{prefix}.mlp.gate_proj.weight", (inter, hidden)),
        (f"{prefix}.mlp.up_proj.weight", (inter, hidden)),
        (f"{prefix}.mlp.down_proj.weight", (hidden, inter)),
        (f"{prefix}.input_layernorm.weight", (hidden,)),
        (f"{prefix}.post_attention_layernorm.weight", (hidden,)),
    ]


def talker_param_specs(cfg: dict):
    """(name, shape) of every talker/code-predictor parameter (M:1427-1445, 1015-1035, 1156-1177, 1564-1586)."""
    t = cfg["talker_config"]
    c = t["code_predictor_config"]
    H, thd = t["hidden_size"], t["text_hidden_size"]
    specs = []
    for i in range(t["num_hidden_layers"]):
        specs += _layer_specs(f"talker.model.layers.{i}", H, t["intermediate_size"], t["num_attention_heads"],
                              t["num_key_value_heads"], t["head_dim"])
    specs += [("talker.model.norm.weight", (H,)),
              ("talker.model.codec_embedding.weight", (t["vocab_size"], H)),
              ("talker.model.text_embedding.weight", (t["text_vocab_size"], thd)),
              ("talker.text_projection.linear_fc1.weight", (thd, thd)),
              ("talker.text_projection.linear_fc1.bias", (thd,)),
              ("talker.text_projection.linear_fc2.weight", (H, thd)),
              ("talker.text_projection.linear_fc2.bias", (H,)),
              ("talker.codec_head.weight", (t["vocab_size"], H))]
    Hc = c["hidden_size"]
    for i in range(c["num_hidden_layers"]):
        specs += _layer_specs(f"talker.code_predictor.model.layers.{i}", Hc, c["intermediate_size"],
                              c["num_attention_heads"], c["num_key_value_heads"], c["head_dim"])
    specs.append(("talker.code_predictor.model.norm.weight", (Hc,)))
    G = t["num_code_groups"]
    for g in range(G - 1):
        specs.append((f"talker.code_predictor.model.codec_embedding.{g}.weight", (c["vocab_size"], H)))
    for g in range(G - 1):
        specs.append((f"talker.code_predictor.lm_head.{g}.weight", (c["vocab_size"], Hc)))
    if Hc != H:
        specs += [("talker.code_predictor.small_to_mtp_projection.weight", (Hc, H)),
                  ("talker.code_predictor.small_to_mtp_projection.bias", (Hc,))]
    return specs


# ----------------------------------------------------------------------------------------------
# building blocks
# ----------------------------------------------------------------------------------------------

def rmsnorm(x: Tensor, w: Tensor, eps: float) -> Tensor:
    """Qwen3TTSRMSNorm (M:595-610): fp32 normalise, cast back, then weight * (two roundings in bf16)."""
    dt = x.dtype
    h = x.to(torch.float32)
    h = h * torch.rsqrt(h.pow(2).mean(-1, keepdim=True) + eps)
    return w * h.to(dt)


def rope_cos_sin(pos: Tensor, head_dim: int, theta: float):
    """Default rope (M:526-592): inv_freq = theta^(-2i/d); emb = cat(f, f); cos/sin in fp32.

    pos: [B, Q] positions (the 3 mrope rows are identical for TTS, so mrope == 1-D rope).
    """
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.int64).float() / head_dim))
    f = pos.float()[..., None] * inv
    emb = torch.cat([f, f], -1)
    return emb.cos(), emb.sin()


def rotate_half(x):
    h = x.shape[-1] // 2
    return torch.cat([-x[..., h:], x[..., :h]], -1)


def apply_rope(x, cos, sin):
    """x [B, nh, Q, D]; cos/sin [B, Q, D] (M:858-882)."""
    return x * cos[:, None] + rotate_half(x) * sin[:, None]


@dataclass
class KV:
    """Per-layer K/V lists; keys [B, nkv, L, D] appended along L (HF DynamicCache.update semantics)."""
    k: List[Optional[Tensor]] = field(default_factory=list)
    v: List[Optional[Tensor]] = field(default_factory=list)

    def update(self, i, k, v):
        while len(self.k) <= i:
            self.k.append(None)
            self.v.append(None)
        if self.k[i] is None:
            self.k[i], self.v[i] = k, v
        else:
            self.k[i] = torch.cat([self.k[i], k], 2)
            self.v[i] = torch.cat([self.v[i], v], 2)
        return self.k[i], self.v[i]

    def length(self):
        return 0 if not self.k or self.k[0] is None else self.k[0].shape[2]


def attention(q, k, v, add_mask, n_rep):
    """eager_attention_forward (M:634-657): repeat_kv, QK^T*scale + mask, softmax in fp32, @V."""
    if n_rep > 1:
        k = k.repeat_interleave(n_rep, dim=1)
        v = v.repeat_interleave(n_rep, dim=1)
    s = torch.matmul(q, k.transpose(2, 3)) * (q.shape[-1] ** -0.5)
    if add_mask is not None:
        s = s + add_mask
    p = torch.softmax(s, -1, dtype=torch.float32).to(q.dtype)
    return torch.matmul(p, v).transpose(1, 2).contiguous()


def decoder_layer(W, pre, x, cos, sin, add_mask, kv: KV, li, lc):
    """Qwen3TTSTalkerDecoderLayer / Qwen3TTSDecoderLayer (M:1348-1424, 961-1012; attention 727-805, 885-958)."""
    B, Q, _ = x.shape
    heads, nkv, hd, eps = lc["num_attention_heads"], lc["num_key_value_heads"], lc["head_dim"], lc["rms_norm_eps"]
    res = x
    h = rmsnorm(x, W[f"{pre}.input_layernorm.weight"], eps)
    q = rmsnorm((h @ W[f"{pre}.self_attn.q_proj.weight"].T).view(B, Q, heads, hd),
                W[f"{pre}.self_attn.q_norm.weight"], eps).transpose(1, 2)
    k = rmsnorm((h @ W[f"{pre}.self_attn.k_proj.weight"].T).view(B, Q, nkv, hd),
                W[f"{pre}.self_attn.k_norm.weight"], eps).transpose(1, 2)
    v = (h @ W[f"{pre}.self_attn.v_proj.weight"].T).view(B, Q, nkv, hd).transpose(1, 2)
    q, k = apply_rope(q, cos, sin), apply_rope(k, cos, sin)
    k, v = kv.update(li, k, v)
    a = attention(q, k, v, add_mask, heads // nkv).reshape(B, Q, heads * hd)
    x = res + a @ W[f"{pre}.self_attn.o_proj.weight"].T
    res = x
    h = rmsnorm(x, W[f"{pre}.post_attention_layernorm.weight"], eps)
    g = F.silu(h @ W[f"{pre}.mlp.gate_proj.weight"].T) * (h @ W[f"{pre}.mlp.up_proj.weight"].T)
    return res + g @ W[f"{pre}.mlp.down_proj.weight"].T


def causal_mask(mask2d: Optional[Tensor], cache_pos: Tensor, kv_len: int, B: int, dtype=torch.float32):
    """4.57 create_causal_mask, eager form: allowed(q,kv) = kv <= cache_pos[q] and mask2d[b,kv]; additive."""
    kv_idx = torch.arange(kv_len)
    allowed = (kv_idx[None, :] <= cache_pos[:, None])[None, None].expand(B, 1, len(cache_pos), kv_len)
    if mask2d is not None:
        allowed = allowed & mask2d[:, None, None, :kv_len].bool()
    m = torch.zeros(allowed.shape, dtype=dtype)
    return m.masked_fill(~allowed, torch.finfo(dtype).min)


# ----------------------------------------------------------------------------------------------
# talker / code predictor forwards
# ----------------------------------------------------------------------------------------------

class TalkerOracle:
    def __init__(self, cfg: dict, weights: Dict[str, Tensor]):
        self.cfg = cfg
        self.t = cfg["talker_config"]
        self.c = self.t["code_predictor_config"]
        self.W = {k: (v if isinstance(v, Tensor) else torch.from_numpy(v)).float() for k, v in weights.items()}

    # --- G1 helpers ---------------------------------------------------------------------------
    def text_proj(self, ids: Tensor) -> Tensor:
        """text_projection(text_embedding(ids)) (M:808-816, 1575-1577): fc2(silu(fc1 x + b1)) + b2."""
        W = self.W
        e = W["talker.model.text_embedding.weight"][ids]
        h = F.silu(e @ W["talker.text_projection.linear_fc1.weight"].T + W["talker.text_projection.linear_fc1.bias"])
        return h @ W["talker.text_projection.linear_fc2.weight"].T + W["talker.text_projection.linear_fc2.bias"]

    def codec_embed(self, ids) -> Tensor:
        if not isinstance(ids, Tensor):
            ids = torch.tensor(ids, dtype=torch.long)
        return self.W["talker.model.codec_embedding.weight"][ids]

    # --- T1-T10 -------------------------------------------------------------------------------
    def talker_forward(self, embeds, mask2d, positions, cache_pos, kv: KV):
        """Qwen3TTSTalkerModel.forward (M:1457-1561) + codec_head (M:1727)."""
        t = self.t
        B = embeds.shape[0]
        cos, sin = rope_cos_sin(positions, t["head_dim"], t["rope_theta"])
        add_mask = causal_mask(mask2d, cache_pos, kv.length() + embeds.shape[1], B)
        x = embeds
        for i in range(t["num_hidden_layers"]):
            x = decoder_layer(self.W, f"talker.model.layers.{i}", x, cos, sin, add_mask, kv, i, t)
        x = rmsnorm(x, self.W["talker.model.norm.weight"], t["rms_norm_eps"])
        return x, x @ self.W["talker.codec_head.weight"].T

    # --- P1-P3 --------------------------------------------------------------------------------
    def cp_forward(self, embeds, kv: KV, gstep: int):
        """CodePredictor forward (M:1250-1312): small_to_mtp_projection -> 5 layers -> norm -> lm_head[g]."""
        c, W = self.c, self.W
        if "talker.code_predictor.small_to_mtp_projection.weight" in W:
            embeds = embeds @ W["talker.code_predictor.small_to_mtp_projection.weight"].T + \
                W["talker.code_predictor.small_to_mtp_projection.bias"]
        B, Q, _ = embeds.shape
        past = kv.length()
        cache_pos = torch.arange(past, past + Q)
        cos, sin = rope_cos_sin(cache_pos[None].expand(B, Q), c["head_dim"], c["rope_theta"])
        add_mask = causal_mask(None, cache_pos, past + Q, B)
        x = embeds
        for i in range(c["num_hidden_layers"]):
            x = decoder_layer(W, f"talker.code_predictor.model.layers.{i}", x, cos, sin, add_mask, kv, i, c)
        x = rmsnorm(x, W["talker.code_predictor.model.norm.weight"], c["rms_norm_eps"])
        return x @ W[f"talker.code_predictor.lm_head.{gstep}.weight"].T

    def cp_generate(self, past_hidden, tok0, sampler):
        """code_predictor.generate(max_new_tokens=G-1) (M:1671-1680): 15 tokens, no EOS/processors."""
        W = self.W
        kv = KV()
        x = torch.cat([past_hidden, self.codec_embed(tok0)[:, None]], 1)
        out = []
        logits = self.cp_forward(x, kv, 0)[:, -1]
        for g in range(self.t["num_code_groups"] - 1):
            tok = sampler(logits.float(), g)
            out.append(tok)
            if g == self.t["num_code_groups"] - 2:
                break
            e = W[f"talker.code_predictor.model.codec_embedding.{g}.weight"][tok][:, None]
            logits = self.cp_forward(e, kv, g + 1)[:, -1]
        return torch.stack(out, 1)

    def frame_embedding(self, tok0, cps):
        """Σ of 16 codebook embeddings (M:1681-1687)."""
        W = self.W
        parts = [self.codec_embed(tok0)[:, None]]
        for i in range(cps.shape[1]):
            parts.append(W[f"talker.code_predictor.model.codec_embedding.{i}.weight"][cps[:, i]][:, None])
        return torch.cat(parts, 1).sum(1, keepdim=True)


# ----------------------------------------------------------------------------------------------
# G1/G2: prompt assembly (M:2068-2269)
# ----------------------------------------------------------------------------------------------

def build_prompts(o: TalkerOracle, input_ids, languages, speakers=None, instruct_ids=None, non_streaming_mode=False,
                  voice_clone_prompt=None, ref_ids=None):
    """Returns (embeds [B,P,H], mask [B,P] int64, trailing [B,T,H], tts_pad_embed [1,1,H]).

    Follows Qwen3TTSForConditionalGeneration.generate prompt construction exactly (M:2068-2269),
    including the dialect override (:2118-2122), speaker splice (:2166-2172), non-streaming text
    layout (:2203-2227), ICL prompt (:1968-2019, 2188-2197) and left padding (:2239-2269).
    """
    cfg, t = o.cfg, o.t
    B = len(input_ids)
    per = [[] for _ in range(B)]
    spk_embeds = None
    if voice_clone_prompt is not None:
        spk_embeds = [torch.as_tensor(e).float() for e in voice_clone_prompt["ref_spk_embedding"]]
    if instruct_ids is not None:
        for i, ins in enumerate(instruct_ids):
            if ins is not None:
                per[i].append(o.text_proj(ins))
    if speakers is None:
        speakers = [None] * B
    trailing = []
    tts_pad = None
    for i, (ids, lang, spk) in enumerate(zip(input_ids, languages, speakers)):
        if spk_embeds is None:
            if spk == "" or spk is None:
                spk_e = None
            else:
                if spk.lower() not in t["spk_id"]:
                    raise NotImplementedError(f"Speaker {spk} not implemented")
                spk_e = o.codec_embed(t["spk_id"][spk.lower()])
        else:
            if voice_clone_prompt["x_vector_only_mode"][i] or voice_clone_prompt["icl_mode"][i]:
                spk_e = spk_embeds[i]
            else:
                spk_e = None
        assert lang is not None
        if lang.lower() == "auto":
            lang_id = None
        else:
            if lang.lower() not in t["codec_language_id"]:
                raise NotImplementedError(f"Language {lang} not implemented")
            lang_id = t["codec_language_id"][lang.lower()]
        if lang.lower() in ["chinese", "auto"] and spk != "" and spk is not None and \
                t["spk_is_dialect"][spk.lower()] is not False:
            lang_id = t["codec_language_id"][t["spk_is_dialect"][spk.lower()]]
        bos_e, eos_e, pad_e = o.text_proj(torch.tensor([[cfg["tts_bos_token_id"], cfg["tts_eos_token_id"],
                                                         cfg["tts_pad_token_id"]]])).chunk(3, dim=1)
        tts_pad = pad_e
        if lang_id is None:
            pre = [t["codec_nothink_id"], t["codec_think_bos_id"], t["codec_think_eos_id"]]
        else:
            pre = [t["codec_think_id"], t["codec_think_bos_id"], lang_id, t["codec_think_eos_id"]]
        c0 = o.codec_embed([pre])
        c1 = o.codec_embed([[t["codec_pad_id"], t["codec_bos_id"]]])
        codec_in = torch.cat([c0, c1], 1) if spk_e is None else torch.cat([c0, spk_e.view(1, 1, -1), c1], 1)
        role = o.text_proj(ids[:, :3])
        body = torch.cat([pad_e.expand(-1, codec_in.shape[1] - 2, -1), bos_e], 1) + codec_in[:, :-1]
        emb = torch.cat([role, body], 1)
        icl = (voice_clone_prompt is not None and voice_clone_prompt["ref_code"] is not None
               and voice_clone_prompt["icl_mode"][i])
        if icl:
            icl_e, trail = _icl_prompt(o, ids[:, 3:-5], ref_ids[i][:, 3:-2],
                                       torch.as_tensor(voice_clone_prompt["ref_code"][i]), pad_e, eos_e,
                                       non_streaming_mode)
            emb = torch.cat([emb, icl_e], 1)
        else:
            emb = torch.cat([emb, o.text_proj(ids[:, 3:4]) + codec_in[:, -1:]], 1)
            if non_streaming_mode:
                emb = emb[:, :-1]
                n = ids[:, 3:-5].shape[1]
                txt = torch.cat([o.text_proj(ids[:, 3:-5]), eos_e], 1) + o.codec_embed([[t["codec_pad_id"]] * (n + 1)])
                emb = torch.cat([emb, txt, pad_e + o.codec_embed([[t["codec_bos_id"]]])], 1)
                trail = pad_e
            else:
                trail = torch.cat([o.text_proj(ids[:, 4:-5]), eos_e], 1)
        per[i].append(emb)
        trailing.append(trail)
    seqs = [torch.cat(p, 1)[0] for p in per]
    P = max(s.shape[0] for s in seqs)
    H = seqs[0].shape[1]
    embeds = torch.zeros(B, P, H)
    mask = torch.zeros(B, P, dtype=torch.long)
    for i, s in enumerate(seqs):
        embeds[i, P - s.shape[0]:] = s
        mask[i, P - s.shape[0]:] = 1
    T = max(tr.shape[1] for tr in trailing)
    trail = tts_pad.squeeze().expand(B, T, H).clone()
    for i, tr in enumerate(trailing):
        trail[i, :tr.shape[1]] = tr[0]
    return embeds, mask, trail, tts_pad


def _icl_prompt(o, text_id, ref_id, ref_code, pad_e, eos_e, non_streaming_mode):
    """generate_icl_prompt (M:1968-2019)."""
    t = o.t
    text = torch.cat([o.text_proj(torch.cat([ref_id, text_id], -1)), eos_e], 1)
    parts = [o.codec_embed(ref_code[:, :1])]
    for i in range(1, t["num_code_groups"]):
        parts.append(o.W[f"talker.code_predictor.model.codec_embedding.{i - 1}.weight"][ref_code[:, i:i + 1]])
    codec = torch.cat(parts, 1).sum(1).unsqueeze(0)
    codec = torch.cat([o.codec_embed([[t["codec_bos_id"]]]), codec], 1)
    tl, cl = text.shape[1], codec.shape[1]
    if non_streaming_mode:
        e = text + o.codec_embed([[t["codec_pad_id"]] * tl])
        return torch.cat([e, codec + pad_e], 1), pad_e
    if tl > cl:
        return text[:, :cl] + codec, text[:, cl:]
    text = torch.cat([text] + [pad_e] * (cl - tl), 1)
    return text + codec, pad_e


# ----------------------------------------------------------------------------------------------
# G3: HF-4.57 GenerationMixin semantics, restated as an explicit loop
# ----------------------------------------------------------------------------------------------

def process_logits(scores, history, n_generated, eos, suppress, rep_penalty, min_new_tokens=2):
    """RepetitionPenalty -> MinNewTokens -> SuppressTokens (transformers 4.57 processor order).

    scores [B,V] fp32; history [B, n] generated tokens (the talker starts from inputs_embeds, so the
    penalised history is the generated ids only).
    """
    scores = scores.clone()
    if rep_penalty != 1.0 and history is not None and history.shape[1] > 0:
        s = torch.gather(scores, 1, history)
        s = torch.where(s < 0, s * rep_penalty, s / rep_penalty)
        scores = scores.scatter(1, history, s)
    if n_generated < min_new_tokens:
        scores[:, eos] = -math.inf
    if suppress:
        scores[:, suppress] = -math.inf
    return scores


def warp_and_sample(scores, temperature, top_k, top_p, gen: torch.Generator):
    """Temperature -> TopK -> TopP warpers, softmax, multinomial (transformers 4.57 sample path)."""
    return torch.multinomial(warp_probs(scores, temperature, top_k, top_p), 1, generator=gen).squeeze(1)


def warp_probs(scores, temperature, top_k, top_p):
    """The distribution warp_and_sample draws from: TemperatureLogitsWarper -> TopKLogitsWarper -> TopPLogitsWarper ->
    softmax (transformers 4.57 `_sample` with do_sample=True)."""
    if temperature is not None and temperature != 1.0:
        scores = scores / temperature
    if top_k is not None and top_k != 0:
        k = min(max(top_k, 1), scores.shape[-1])
        kth = torch.topk(scores, k)[0][..., -1, None]
        scores = scores.masked_fill(scores < kth, -math.inf)
    if top_p is not None and top_p < 1.0:
        sl, si = torch.sort(scores, descending=False)
        cp = sl.softmax(-1).cumsum(-1)
        rm = cp <= (1 - top_p)
        rm[..., -1:] = 0
        scores = scores.masked_fill(rm.scatter(1, si, rm), -math.inf)
    return torch.softmax(scores, -1)


@dataclass
class GenResult:
    codes: List[Tensor]          # per item [F_i, 16] int64
    hidden: List[Tensor]         # per item [F_i, H]
    raw_tokens: Tensor           # [B, n] sampled cb0 tokens
    logits0: Optional[Tensor] = None  # processed prefill scores (debug)
    margins: Optional[List[float]] = None  # greedy top-2 margins of every argmax taken (talker + CP)


def generate(o: TalkerOracle, embeds, mask, trailing, tts_pad, max_new_tokens=4096, do_sample=False, top_k=50,
             top_p=1.0, temperature=0.9, subtalker_dosample=False, subtalker_top_k=50, subtalker_top_p=1.0,
             subtalker_temperature=0.9, eos_token_id=None, repetition_penalty=1.05, ignore_eos=False,
             seed=0, record_margins=False) -> GenResult:
    """Qwen3TTSForConditionalGeneration.generate's talker.generate + post-processing (M:2044-2066, 2272-2292).

    `ignore_eos` adds EOS to the suppress set (benchmark mode: fixed frame count)."""
    t = o.t
    V = t["vocab_size"]
    eos = eos_token_id if eos_token_id is not None else t["codec_eos_token_id"]
    suppress = [i for i in range(V - 1024, V) if i != t["codec_eos_token_id"]]
    if ignore_eos:
        suppress = suppress + [eos]
    gen = torch.Generator().manual_seed(seed)
    margins = [] if record_margins else None

    def pick(scores, sample, tk, tp, temp):
        if sample:
            return warp_and_sample(scores, temp, tk, tp, gen)
        if margins is not None:
            top2 = torch.topk(scores, 2, -1)[0]
            margins.extend((top2[:, 0] - top2[:, 1]).tolist())
        return torch.argmax(scores, -1)

    B, P, H = embeds.shape
    kv = KV()
    # prefill positions: get_rope_index (M:1746-1800) + rope_deltas (M:1693-1704)
    pos = mask.float().cumsum(-1) - 1
    pos = pos.masked_fill(mask == 0, 1)
    max_pos = pos.max(-1, keepdim=True)[0]
    rope_deltas = (max_pos + 1 - mask.sum(-1, keepdim=True)) - (1 - mask).sum(-1, keepdim=True)
    hidden, logits = o.talker_forward(embeds, mask, pos.long(), torch.arange(P), kv)
    past_hidden = hidden[:, -1:]
    tokens, codes, hiddens = [], [], []
    unfinished = torch.ones(B, dtype=torch.bool)
    attn_mask = mask.clone()
    step = 0
    while True:
        scores = process_logits(logits[:, -1].float(), torch.stack(tokens, 1) if tokens else None, len(tokens),
                                eos, suppress, repetition_penalty)
        nxt = pick(scores, do_sample, top_k, top_p, temperature)
        nxt = torch.where(unfinished, nxt, torch.full_like(nxt, eos))
        tokens.append(nxt)
        unfinished = unfinished & (nxt != eos)
        if (not unfinished.any()) or len(tokens) >= max_new_tokens:
            break
        # decode step (M:1669-1744)
        hiddens.append(past_hidden[:, 0])
        cps = o.cp_generate(past_hidden, nxt,
                            lambda lg, g: pick(lg, subtalker_dosample, subtalker_top_k, subtalker_top_p,
                                               subtalker_temperature))
        codes.append(torch.cat([nxt[:, None], cps], 1))
        e = o.frame_embedding(nxt, cps)
        e = e + (trailing[:, step:step + 1] if step < trailing.shape[1] else tts_pad)
        attn_mask = torch.cat([attn_mask, torch.ones(B, 1, dtype=attn_mask.dtype)], 1)
        cache_pos = torch.tensor([P + step])
        positions = (cache_pos[0] + rope_deltas).long()  # [B,1] (M:1705-1711)
        hidden, logits = o.talker_forward(e, attn_mask, positions, cache_pos, kv)
        past_hidden = hidden[:, -1:]
        step += 1
    raw = torch.stack(tokens, 1)
    if codes:
        all_codes = torch.stack(codes, 1)
        all_hidden = torch.stack(hiddens, 1)
    else:
        all_codes = torch.zeros(B, 0, t["num_code_groups"], dtype=torch.long)
        all_hidden = torch.zeros(B, 0, H)
    first = all_codes[:, :, 0]
    is_stop = first == t["codec_eos_token_id"]
    stop_idx = torch.argmax(is_stop.int(), 1) if all_codes.shape[1] else torch.zeros(B, dtype=torch.long)
    eff = torch.where(is_stop.any(1), stop_idx, torch.full_like(stop_idx, all_codes.shape[1]))
    return GenResult([all_codes[i, :eff[i]] for i in range(B)], [all_hidden[i, :eff[i]] for i in range(B)], raw,
                     margins=margins)
