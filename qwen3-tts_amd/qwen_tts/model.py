"""`Qwen3TTSForConditionalGeneration` equivalent on the MI355X engine (inner generate() contract).

Prompt assembly follows qwen_tts/core/models/modeling_qwen3_tts.py (M) :1968-2269 exactly; every
embedding / text-projection product runs through the HIP kernels (gather + fused MFMA GEMMs), the
sequence layout (cat / left-pad) is torch plumbing on device tensors.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import torch

from . import kernels as K
from .talker import MIN_NEW_TOKENS, GenParams, HandoffWatch, TalkerEngine


class _Runs:
    """Runs of text ids / codec ids collected for one batched text_projection + one codec-embedding gather."""

    def __init__(self):
        self.ids = {"t": [], "c": []}
        self.out = {}

    def _add(self, kind, ids):
        ids = [int(x) for x in (ids.reshape(-1).tolist() if isinstance(ids, torch.Tensor) else ids)]
        s = len(self.ids[kind])
        self.ids[kind].extend(ids)
        return kind, s, len(ids)

    def text(self, ids):
        return self._add("t", ids)

    def codec(self, ids):
        return self._add("c", ids)

    def run(self, e):
        if self.ids["t"]:
            self.out["t"] = e.text_proj(self.ids["t"])
        if self.ids["c"]:
            self.out["c"] = e.codec_embed(self.ids["c"])

    def get(self, h):
        kind, s, n = h
        return self.out[kind][s:s + n][None]


class TTSModel:
    def __init__(self, config: dict, weights: Dict[str, torch.Tensor], dtype="bf16", device="cuda",
                 generate_config: Optional[dict] = None):
        self.config = config
        self.tc = config["talker_config"]
        self.engine = TalkerEngine(config, weights, dtype=dtype, device=device)
        self.device = self.engine.dev
        self.tts_model_type = config.get("tts_model_type")
        self.tts_model_size = config.get("tts_model_size")
        self.tokenizer_type = config.get("tokenizer_type")
        self.generate_config = generate_config or {}
        self.speech_tokenizer = None
        self.supported_speakers = list((self.tc.get("spk_id") or {}).keys())
        self.supported_languages = ["auto"] + [k for k in (self.tc.get("codec_language_id") or {}) if "dialect" not in k]
        self.speaker_encoder_sample_rate = config.get("speaker_encoder_config", {}).get("sample_rate", 24000)
        self.speaker_encoder = None
        if self.tts_model_type == "base" and "speaker_encoder.fc.weight" in weights:  # M:1821-1824
            from .speaker import SpeakerEncoder
            self.speaker_encoder = SpeakerEncoder(config, weights, dtype=dtype, device=self.device)

    @torch.inference_mode()
    def extract_speaker_embedding(self, audio, sr):
        """M:1940-1954: 24 kHz mono float32 waveform -> x-vector [enc_dim] (device, fp32)."""
        assert sr == 24000, "Only support 24kHz audio"
        if self.speaker_encoder is None:
            raise ValueError("no speaker encoder loaded (tts_model_type != 'base', or its weights are absent)")
        with torch.cuda.device(self.device):
            return self.speaker_encoder.embed(audio)

    @torch.inference_mode()
    def extract_speaker_embeddings(self, audios, sr):
        """extract_speaker_embedding of several clips at once (equal-length clips share one ECAPA pass):
        [n][enc_dim] (device, fp32)."""
        assert sr == 24000, "Only support 24kHz audio"
        if self.speaker_encoder is None:
            raise ValueError("no speaker encoder loaded (tts_model_type != 'base', or its weights are absent)")
        with torch.cuda.device(self.device):
            return self.speaker_encoder.embed_many(audios)

    def get_supported_speakers(self):
        return self.supported_speakers

    def get_supported_languages(self):
        return self.supported_languages

    def load_speech_tokenizer(self, tok):
        self.speech_tokenizer = tok

    # -------------------------------------------------------------------------------- G1 / G2
    def _icl_prompt(self, text_id, ref_id, ref_code, pad_e, eos_e, non_streaming_mode):
        """generate_icl_prompt (M:1968-2019)."""
        e, t = self.engine, self.tc
        text = torch.cat([e.text_proj(torch.cat([ref_id, text_id], -1))[None], eos_e], 1)
        ref_code = ref_code.to(self.device)
        parts = [e.codec_embed(ref_code[:, 0])]
        for i in range(1, t["num_code_groups"]):
            parts.append(e.cp_embed(i - 1, ref_code[:, i]))
        codec = torch.stack(parts, 1).sum(1)[None]
        codec = torch.cat([e.codec_embed([t["codec_bos_id"]])[None], codec], 1)
        tl, cl = text.shape[1], codec.shape[1]
        if non_streaming_mode:
            x = text + e.codec_embed([t["codec_pad_id"]] * tl)[None]
            return torch.cat([x, codec + pad_e], 1), pad_e
        if tl > cl:
            return text[:, :cl] + codec, text[:, cl:]
        text = torch.cat([text] + [pad_e] * (cl - tl), 1)
        return text + codec, pad_e

    def build_prompts(self, input_ids, languages, speakers=None, instruct_ids=None, non_streaming_mode=False,
                      voice_clone_prompt=None, ref_ids=None):
        """(embeds [B,P,H] fp32, mask [B,P], trailing [B,T,H], tts_pad [1,1,H]) -- M:2068-2269.
        Two passes: the rows' text-id and codec-id runs are collected on the host first, then projected in one
        text_projection and one codec-embedding gather for the whole batch (one host->device copy each instead of
        a few per row: the per-row calls were host-bound, ~3.3 ms at B=8), and each row is assembled from slices."""
        e, t, cfg = self.engine, self.tc, self.config
        B = len(input_ids)
        runs = _Runs()
        spk_embeds = None
        if voice_clone_prompt is not None:
            spk_embeds = [torch.as_tensor(x).to(self.device).float() for x in voice_clone_prompt["ref_spk_embedding"]]
        h_ins = [None] * B
        if instruct_ids is not None:
            for i, ins in enumerate(instruct_ids):
                if ins is not None:
                    h_ins[i] = runs.text(ins)
        if speakers is None:
            speakers = [None] * B
        h_special = runs.text([cfg["tts_bos_token_id"], cfg["tts_eos_token_id"], cfg["tts_pad_token_id"]])
        plans = []
        for i, (ids, lang, spk) in enumerate(zip(input_ids, languages, speakers)):
            ids = torch.as_tensor(ids).reshape(-1).tolist()
            pl = {"ids": ids}
            spk_e = None
            if spk_embeds is None:
                if spk == "" or spk is None:
                    pass
                else:
                    if spk.lower() not in t["spk_id"]:
                        raise NotImplementedError(f"Speaker {spk} not implemented")
                    pl["spk_code"] = runs.codec([t["spk_id"][spk.lower()]])
            else:
                use = voice_clone_prompt["x_vector_only_mode"][i] or voice_clone_prompt["icl_mode"][i]
                spk_e = spk_embeds[i] if use else None
            pl["spk_vec"] = spk_e
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
            if lang_id is None:
                pre = [t["codec_nothink_id"], t["codec_think_bos_id"], t["codec_think_eos_id"]]
            else:
                pre = [t["codec_think_id"], t["codec_think_bos_id"], lang_id, t["codec_think_eos_id"]]
            pl["c0"] = runs.codec(pre)
            pl["c1"] = runs.codec([t["codec_pad_id"], t["codec_bos_id"]])
            pl["role"] = runs.text(ids[:3])
            pl["icl"] = (voice_clone_prompt is not None and voice_clone_prompt["ref_code"] is not None
                         and voice_clone_prompt["icl_mode"][i])
            if not pl["icl"]:
                pl["first"] = runs.text(ids[3:4])
                if non_streaming_mode:
                    n = len(ids[3:-5])
                    pl["txt"] = runs.text(ids[3:-5])
                    pl["txt_pad"] = runs.codec([t["codec_pad_id"]] * (n + 1))
                    pl["end_bos"] = runs.codec([t["codec_bos_id"]])
                else:
                    pl["trail"] = runs.text(ids[4:-5])
            plans.append(pl)
        runs.run(e)
        if not any(pl["icl"] for pl in plans):
            return self._assemble_indexed(runs, plans, h_ins, h_special, non_streaming_mode)
        special = runs.get(h_special)[0]
        bos_e, eos_e, pad_e = special[0].view(1, 1, -1), special[1].view(1, 1, -1), special[2].view(1, 1, -1)
        per: List[list] = [[] if h_ins[i] is None else [runs.get(h_ins[i])] for i in range(B)]
        trailing = []
        for i, pl in enumerate(plans):
            c0, c1 = runs.get(pl["c0"]), runs.get(pl["c1"])
            spk_e = runs.get(pl["spk_code"]) if "spk_code" in pl else pl["spk_vec"]
            codec_in = torch.cat([c0, c1], 1) if spk_e is None else torch.cat([c0, spk_e.view(1, 1, -1), c1], 1)
            role = runs.get(pl["role"])
            body = torch.cat([pad_e.expand(-1, codec_in.shape[1] - 2, -1), bos_e], 1) + codec_in[:, :-1]
            emb = torch.cat([role, body], 1)
            if pl["icl"]:
                ids = torch.as_tensor(pl["ids"]).reshape(1, -1)
                ref = torch.as_tensor(ref_ids[i]).reshape(1, -1)
                icl_e, trail = self._icl_prompt(ids[:, 3:-5], ref[:, 3:-2],
                                                torch.as_tensor(voice_clone_prompt["ref_code"][i]), pad_e, eos_e,
                                                non_streaming_mode)
                emb = torch.cat([emb, icl_e], 1)
            else:
                emb = torch.cat([emb, runs.get(pl["first"]) + codec_in[:, -1:]], 1)
                if non_streaming_mode:
                    emb = emb[:, :-1]
                    txt = torch.cat([runs.get(pl["txt"]), eos_e], 1) + runs.get(pl["txt_pad"])
                    emb = torch.cat([emb, txt, pad_e + runs.get(pl["end_bos"])], 1)
                    trail = pad_e
                else:
                    trail = torch.cat([runs.get(pl["trail"]), eos_e], 1)
            per[i].append(emb)
            trailing.append(trail)
        seqs = [torch.cat(p, 1)[0] for p in per]
        P = max(s.shape[0] for s in seqs)
        H = seqs[0].shape[1]
        embeds = torch.zeros(B, P, H, device=self.device)
        mask = torch.zeros(B, P, dtype=torch.long, device=self.device)
        for i, s in enumerate(seqs):
            embeds[i, P - s.shape[0]:] = s
            mask[i, P - s.shape[0]:] = 1
        T = max(tr.shape[1] for tr in trailing)
        trail = pad_e.reshape(1, 1, H).expand(B, T, H).clone()
        for i, tr in enumerate(trailing):
            trail[i, :tr.shape[1]] = tr[0]
        return embeds, mask, trail, pad_e

    def _assemble_indexed(self, runs, plans, h_ins, h_special, non_streaming_mode):
        """build_prompts' assembly for non-ICL rows as one gather: every prompt / trailing position is the sum of at
        most two rows of [text projections; codec embeddings; x-vectors; zero row], so the host writes a [positions,
        2] index table and three GPU ops build the whole batch (the per-row slicing / cat / add chain was ~120
        host-bound launches at B = 8).  Same two fp32 operands per position as that chain, so the same bits."""
        B = len(plans)
        out_t, out_c = runs.out.get("t"), runs.out.get("c")
        NT = 0 if out_t is None else out_t.shape[0]
        NC = 0 if out_c is None else out_c.shape[0]
        vecs = [pl["spk_vec"] for pl in plans if pl["spk_vec"] is not None]
        Z = NT + NC + len(vecs)  # the zero row

        def t(h, j=0):
            return h[1] + j

        def c(h, j=0):
            return NT + h[1] + j
        sp = h_special
        bos, eos, pad = t(sp, 0), t(sp, 1), t(sp, 2)
        seqs, trails, v = [], [], 0
        for i, pl in enumerate(plans):
            pos = [] if h_ins[i] is None else [(t(h_ins[i], j), Z) for j in range(h_ins[i][2])]
            pos += [(t(pl["role"], j), Z) for j in range(3)]
            ci = [c(pl["c0"], j) for j in range(pl["c0"][2])]
            if "spk_code" in pl:
                ci.append(c(pl["spk_code"]))
            elif pl["spk_vec"] is not None:
                ci.append(NT + NC + v)
                v += 1
            ci += [c(pl["c1"], j) for j in range(2)]
            pos += [(pad if k < len(ci) - 2 else bos, ci[k]) for k in range(len(ci) - 1)]
            if non_streaming_mode:
                n = pl["txt"][2]
                pos += [(t(pl["txt"], j) if j < n else eos, c(pl["txt_pad"], j)) for j in range(n + 1)]
                pos.append((pad, c(pl["end_bos"])))
                trails.append([(pad, Z)])
            else:
                if pl["first"][2]:  # (a prompt without a first text token has no such position, as in the chain)
                    pos.append((t(pl["first"]), ci[-1]))
                trails.append([(t(pl["trail"], j), Z) for j in range(pl["trail"][2])] + [(eos, Z)])
            seqs.append(pos)
        P, T = max(len(s) for s in seqs), max(len(tr) for tr in trails)
        idx = [[(Z, Z)] * (P - len(s)) + s for s in seqs] + [tr + [(pad, Z)] * (T - len(tr)) for tr in trails]
        H = (out_t if out_t is not None else out_c).shape[1]
        parts = [x for x in (out_t, out_c) if x is not None] + [x.reshape(1, H) for x in vecs] + \
            [torch.zeros(1, H, device=self.device)]
        table = torch.cat(parts, 0)
        ix = torch.tensor([p for row in idx for p in row], dtype=torch.long).pin_memory().to(self.device,
                                                                                             non_blocking=True)
        rows = table[ix.view(-1)].view(-1, 2, H).sum(1)
        embeds = rows[:B * P].view(B, P, H)
        trail = rows[B * P:].view(B, T, H)
        mask = torch.tensor([[0] * (P - len(s)) + [1] * len(s) for s in seqs], dtype=torch.long).pin_memory().to(
            self.device, non_blocking=True)
        pad_e = table[pad].view(1, 1, H)
        return embeds, mask, trail, pad_e

    # -------------------------------------------------------------------------------- generate
    @torch.no_grad()
    def generate(self, input_ids=None, instruct_ids=None, ref_ids=None, voice_clone_prompt=None, languages=None,
                 speakers=None, non_streaming_mode=False, max_new_tokens=4096, do_sample=True, top_k=50, top_p=1.0,
                 temperature=0.9, subtalker_dosample=True, subtalker_top_k=50, subtalker_top_p=1.0,
                 subtalker_temperature=0.9, eos_token_id=None, repetition_penalty=1.05, ignore_eos=False, seed=None,
                 use_graph=True, max_batch=None, philox_ids=None, frame_caps=None, **kwargs):
        """Same contract as Qwen3TTSForConditionalGeneration.generate (M:2022-2292):
        returns (list of [F_i,16] int64 codes, list of [F_i,H] last hidden states).

        philox_ids (not in the reference): the sampling stream id of each request (default its index in this call);
        the data-parallel runner (qwen_tts.dp.dp_generate) passes global request indices.  frame_caps (not in the
        reference): per-request frame limits below max_new_tokens - 1 (decoded through serve()).

        max_batch (not in the reference): with more requests than max_batch, decode them by continuous batching
        through max_batch batch rows (TalkerEngine.serve: a row is refilled with the next request as soon as its
        request ends).  Per request the result is that of the one-shot batched call (same Philox stream per request
        index; per-row arithmetic does not depend on the batch's other rows)."""
        emb, mask, trail, pad = self.build_prompts(input_ids, languages, speakers, instruct_ids, non_streaming_mode,
                                                   voice_clone_prompt, ref_ids)
        gp = GenParams(max_new_tokens, do_sample, top_k, top_p, temperature, subtalker_dosample, subtalker_top_k,
                       subtalker_top_p, subtalker_temperature, eos_token_id, repetition_penalty, ignore_eos, seed)
        B, P = emb.shape[0], emb.shape[1]
        if (max_batch is not None and B > int(max_batch)) or frame_caps is not None:
            n_real = mask.sum(-1).tolist()
            reqs = [(emb[i, P - int(n_real[i]):], trail[i], None if frame_caps is None else frame_caps[i])
                    for i in range(B)]
            max_batch = B if max_batch is None else max_batch
            codes, hid = [None] * B, [None] * B
            for i, c, h in self.engine.serve(reqs, pad, gp, slots=int(max_batch), use_graph=use_graph,
                                             philox_ids=philox_ids):
                codes[i], hid[i] = c, h
            return codes, hid
        return self.engine.generate_from_embeds(emb, mask, trail, pad, gp, use_graph=use_graph, philox_ids=philox_ids)

    @torch.no_grad()
    def teacher_forced(self, ref_codes, input_ids=None, instruct_ids=None, ref_ids=None, voice_clone_prompt=None,
                       languages=None, speakers=None, non_streaming_mode=False, repetition_penalty=1.05,
                       eos_token_id=None, use_graph=True, **kwargs):
        """Greedy choices of this path at every step of the reference's own code sequence (parity diagnostics; not in
        the reference): the prompt is assembled as generate() does, each talker / code-predictor argmax is recorded
        and then replaced by the reference token of ref_codes (list of [F_b, 16]).  Returns (picks [B, F, 16], hidden
        [B, F, H]) so a bf16 run can be compared with fp32 reference codes position by position."""
        emb, mask, trail, pad = self.build_prompts(input_ids, languages, speakers, instruct_ids, non_streaming_mode,
                                                   voice_clone_prompt, ref_ids)
        gp = GenParams(max_new_tokens=2, do_sample=False, subtalker_dosample=False, eos_token_id=eos_token_id,
                       repetition_penalty=repetition_penalty)
        return self.engine.teacher_forced(emb, mask, trail, pad, gp, ref_codes, use_graph=use_graph)

    # -------------------------------------------------------------------------------- streaming
    REF_CHUNK, REF_CTX = 300, 25  # Qwen3TTSTokenizerV2Decoder.chunked_decode (K:885-895)

    @torch.no_grad()
    def stream(self, input_ids=None, instruct_ids=None, ref_ids=None, voice_clone_prompt=None, languages=None,
               speakers=None, non_streaming_mode=False, max_new_tokens=4096, do_sample=True, top_k=50, top_p=1.0,
               temperature=0.9, subtalker_dosample=True, subtalker_top_k=50, subtalker_top_p=1.0,
               subtalker_temperature=0.9, eos_token_id=None, repetition_penalty=1.05, ignore_eos=False, seed=None,
               first_chunk_frames=1, chunk_frames=48, left_context=None, use_graph=True, **kwargs):
        """Streaming generation (the reference has none): yields (row, pcm, last) as frames finish.

        Per row the chunks concatenate to the one-shot generate() + decode() PCM (Z:259-365): the reference
        decodes the zero-right-padded batch in 300-frame chunks with 25 frames of left context, dropping the
        last 555 samples of each chunk (no next frame), and keeps 1920 x #nonzero-cb0 samples.  Default
        (left_context=None): one stateful incremental decoder per reference chunk (codec.CodecStream, primed with the
        chunk's 25 context frames) is fed each final frame once and every sample computable so far is emitted (a
        chunk yields 1920 n - 555 samples after its n frames: no lookahead frame is waited for), so every sample is
        computed once and equals the one-shot output up to fp summation order.  An int `left_context` selects the
        stateless form instead (windows [s, e) within a reference chunk, one lookahead frame), re-decoded from
        min(its chunk's start, left_context frames back) -- 325 reproduces the reference, less is approximate (in
        fp32 150 frames -> rel-L2 1e-6, 72 -> 7e-4, 25 -> 2e-2; tools/stream_fidelity.py).  Codes are identical to
        generate().  pcm is a 1-D fp32 device tensor of 24 kHz samples."""
        dec = self.speech_tokenizer.model
        up = dec.total_upsample
        RC, RX = self.REF_CHUNK, self.REF_CTX
        refs = voice_clone_prompt.get("ref_code") if voice_clone_prompt is not None else None
        prefix = None if refs is None or all(r is None for r in refs) else list(refs)
        # voice clone: the reference frames every row starts with are known at submit -- their codec decode starts on
        # a side stream before the (host-bound) prompt assembly, so it runs beside it instead of beside the prefill
        started = self._start_ref_decode(dec, prefix, len(prefix)) if prefix is not None and left_context is None \
            else None
        try:
            emb, mask, trail, pad = self.build_prompts(input_ids, languages, speakers, instruct_ids,
                                                       non_streaming_mode, voice_clone_prompt, ref_ids)
            gp = GenParams(max_new_tokens, do_sample, top_k, top_p, temperature, subtalker_dosample, subtalker_top_k,
                           subtalker_top_p, subtalker_temperature, eos_token_id, repetition_penalty, ignore_eos, seed)
        except BaseException:
            # the side-stream reference decode holds a pooled codec slot: hand it back before the error propagates
            if started is not None:
                torch.cuda.current_stream(self.device).wait_stream(started[1])
                started[2].close()
            raise
        eos = self.engine.tc["codec_eos_token_id"]
        B = emb.shape[0]
        emitted = 0                       # windows [0, emitted) decoded for every row
        end = [None] * B                  # frame count of each row once its EOS is seen
        cap = [None] * B                  # one-shot sample count (1920 x #nonzero cb0) once the row has ended
        done = [False] * B
        cum = [0] * B                     # samples emitted per row
        # chunk sizes double from first_chunk_frames up to chunk_frames: each chunk's audio (80 ms per frame) covers
        # the generation of the next one (~3 ms per frame), so playback started at the first packet never starves
        if left_context is None:
            yield from self._stream_stateful(dec, emb, mask, trail, pad, gp, B, eos, first_chunk_frames, chunk_frames,
                                             use_graph, prefix, started)
            return
        if prefix is not None:
            raise NotImplementedError("stream(left_context=...) with voice-clone reference codes (ICL): use the "
                                      "default stateful stream")
        it = self.engine.decode_iter(emb, mask, trail, pad, gp, use_graph=use_graph, every=chunk_frames,
                                     first=first_chunk_frames + 1, grow=True)
        for sessions, frames, final in it:
            # codes of frames [0, frames) are final; column `frames` holds the next cb0 (EOS of finishing rows)
            codes = torch.cat([s.codes[:, :frames + 1] for s in sessions], 0)  # int32 [B, frames+1, 16], device
            c0 = codes[:, :, 0].cpu()
            if not final and sessions[0].watch is not None:  # (synchronised above) before any audio is handed out
                sessions[0].watch.check()
            for b in range(B):
                if end[b] is None:
                    hit = (c0[b, emitted:] == eos).nonzero()
                    if hit.numel():
                        end[b] = emitted + int(hit[0])
                if final and end[b] is None:
                    end[b] = frames
                if end[b] is not None and cap[b] is None:
                    cap[b] = up * int((c0[b, :end[b]] != 0).sum())
            # the batch's length once known: every row ended (longest row), or generation stopped
            t_end = max(end) if all(x is not None for x in end) else None
            target = t_end if t_end is not None else frames - 1  # else keep frame `frames-1` as lookahead
            while emitted < target:
                k = emitted // RC
                cend = (k + 1) * RC
                e = min(target, cend)
                closed = e == cend or e == t_end  # this reference chunk ends at e
                base = k * RC - (RX if k * RC - RX > 0 else k * RC)
                hi = e if closed else e + 1
                ctx = min(emitted - base, left_context)
                lo = emitted - ctx
                cc = codes[:, lo:hi].clone()
                for b in range(B):  # finished rows continue as the one-shot batch decode's zero padding
                    if end[b] is not None and end[b] < hi:
                        cc[b, max(end[b] - lo, 0):] = 0
                w = dec.forward(cc)
                n = up * (e - emitted) - (555 if closed else 0)
                for b in range(B):
                    if done[b]:
                        continue
                    take = n if cap[b] is None else max(0, min(n, cap[b] - cum[b]))
                    chunk = w[b, ctx * up:ctx * up + take]
                    cum[b] += take
                    last = cap[b] is not None and (cum[b] >= cap[b] or e == t_end)
                    done[b] = last
                    yield b, chunk, last
                emitted = e
            if t_end is not None and emitted >= t_end:
                for b in range(B):  # rows whose output was complete before the last window
                    if not done[b]:
                        done[b] = True
                        yield b, torch.zeros(0, device=codes.device), True
            if all(done):
                break

    @staticmethod
    def _stream_window(codes, pre, R, end, lo, hi):
        """Decode positions [lo, hi) of every row's sequence prefix_b + generated_b + zeros, int32 [B, hi-lo, 16]
        (generated frame f of row b sits at position R_b + f; rows past their end are the batch decode's zero
        padding)."""
        B = codes.shape[0]
        if not any(R):
            cc = codes[:, lo:hi].clone()
            for b in range(B):
                if end[b] is not None and end[b] < hi:
                    cc[b, max(end[b] - lo, 0):] = 0
            return cc
        cc = torch.zeros(B, hi - lo, codes.shape[2], dtype=codes.dtype, device=codes.device)
        for b in range(B):
            if R[b] > lo:  # prefix part
                cc[b, :min(R[b], hi) - lo] = pre[b][lo:min(R[b], hi)]
            g0, g1 = max(lo, R[b]) - R[b], hi - R[b]  # generated frames [g0, g1)
            if end[b] is not None:
                g1 = min(g1, end[b])
            if g1 > g0:
                cc[b, g0 + R[b] - lo:g1 + R[b] - lo] = codes[b, g0:g1]
        return cc

    def _start_ref_decode(self, dec, prefix, B):
        """Feed every row's leading reference frames (the first min(R_b, 300) of them) to a fresh incremental decoder
        on a side stream; returns (pre, side stream, decoder, frames fed) for _stream_stateful, or None when some row
        has no reference frames."""
        dev = self.device
        pre = [None if x is None else torch.as_tensor(x).to(dev, torch.int32) for x in prefix]
        if any(x is None or x.shape[0] == 0 for x in pre):
            return None
        main = torch.cuda.current_stream(dev)
        side = K.side_stream(dev)
        side.wait_stream(main)
        with torch.cuda.stream(side):  # (the stream's state slot brings its own split-K workspace)
            cs = dec.stream(B, self.REF_CTX + self.REF_CHUNK)
            fed = min(min(int(x.shape[0]) for x in pre), self.REF_CHUNK)
            cs.feed(torch.stack([x[:fed] for x in pre]))
        return pre, side, cs, fed

    def _stream_stateful(self, dec, emb, mask, trail, pad, gp, B, eos, first_chunk_frames, chunk_frames, use_graph,
                         prefix=None, started=None):
        """stream() on the incremental codec: every final frame is fed once to the decoder of its reference chunk
        and every sample computable from the frames fed so far is emitted -- 1920 n - 555 samples of a chunk after
        its n frames, i.e. no lookahead frame is waited for (the 555 samples that need it follow with the next
        chunk; at a reference chunk's end they are dropped, as the reference's chunked decode drops them).

        prefix[b] (voice clone, ICL mode): the reference codes int [R_b, 16] that generate_voice_clone decodes in
        front of row b's generated codes (W:263-274, `cat(ref_code, codes)` then a proportional cut).  Row b's decode
        sequence is then ref_b + generated + zero padding; the ref frames are known at submit and fed with the first
        chunk, and row b's output starts at sample 1920 R_b of its sequence, the reference/generated boundary.  The
        wrapper's proportional cut int(R_b / T_b * len_b) lands floor(555 R_b / T_b) samples earlier (len_b lacks
        the last frame's 555 lookahead samples), at a point that depends on the final length T_b, which a stream
        does not know when it starts: the streamed PCM is generate_voice_clone's PCM without those leading samples
        (< 555, e.g. 72 for 38 reference frames + 256 generated)."""
        up = dec.total_upsample
        RC, RX = self.REF_CHUNK, self.REF_CTX
        dev = self.device
        if started is not None:
            pre = started[0]
        else:
            pre = [None] * B if prefix is None else [None if x is None else torch.as_tensor(x).to(dev, torch.int32)
                                                      for x in prefix]
        R = [0 if x is None else int(x.shape[0]) for x in pre]
        pre_nz = [0 if x is None else int((x[:, 0] != 0).sum()) for x in pre]
        end = [None] * B                  # generated frame count of each row once its EOS is seen
        cap = [None] * B                  # one-shot sample count (1920 x #nonzero cb0 of its sequence) once ended
        done = [False] * B
        skip = [up * r for r in R]        # samples of row b's sequence before its output starts
        gpos = 0                          # samples of the (shared) decode timeline produced so far
        scanned = 0                       # cb0 columns already searched for EOS
        k, cs, fed, emit_s, ctx_s = 0, None, 0, 0, 0   # reference chunk, its decoder, positions fed, samples emitted
        main, side = torch.cuda.current_stream(dev), None
        if started is not None:  # stream() began decoding the reference frames before the prompt assembly
            _, side, cs, fed = started
        elif min(R) > 0:
            # every row starts with reference frames, known at submit: decode them on a side stream while the talker
            # prefills and generates the first frames on this one
            _, side, cs, fed = self._start_ref_decode(dec, pre, B)
        # a one-frame first chunk is handed over as soon as frame 0's codes exist: its codec window is queued before the
        # talker step that starts frame 1 (the first packet does not wait for it)
        it = self.engine.decode_iter(emb, mask, trail, pad, gp, use_graph=use_graph, every=chunk_frames,
                                     first=first_chunk_frames, grow=True, early_first=first_chunk_frames == 1)
        try:
            for sessions, frames, final in it:
                if side is not None:
                    main.wait_stream(side)
                    side = None
                # codes of frames [0, frames) are final; column `frames` holds the next cb0 (EOS of finishing rows)
                codes = torch.cat([s.codes[:, :frames + 1] for s in sessions], 0)  # int32 [B, frames+1, 16], device
                # the EOS scan reads cb0 on the host (a sync on the frame just launched); columns [0, frames] hold
                # tokens sampled at n_generated <= frames, and EOS is suppressed below MIN_NEW_TOKENS, so the first
                # chunk skips the scan and its codec feed is queued right behind the frame
                # frames not covered by a watch check yet (the early first chunk skips the scan): checked, behind their
                # codec feed, before the first of their audio is handed out
                unchecked = not (final or frames + 1 > MIN_NEW_TOKENS)
                if not unchecked:
                    c0 = codes[:, :, 0].cpu()
                    for b in range(B):
                        if end[b] is None:
                            hit = (c0[b, scanned:] == eos).nonzero()
                            if hit.numel():
                                end[b] = scanned + int(hit[0])
                        if final and end[b] is None:
                            end[b] = frames
                        if end[b] is not None and cap[b] is None:
                            cap[b] = up * (pre_nz[b] + int((c0[b, :end[b]] != 0).sum()))
                    scanned = frames
                    # the host just synchronised on these frames: a hand-off give-up among them raises before any
                    # of their audio is handed out
                    if sessions[0].watch is not None:
                        sessions[0].watch.check()
                # decode positions (prefix + generated) available for every row; the sequence length once all ended
                t_end = max(R[b] + end[b] for b in range(B)) if all(x is not None for x in end) else None
                avail = t_end if t_end is not None else min(R[b] + frames for b in range(B) if end[b] is None)
                while True:
                    cend = (k + 1) * RC
                    if cs is None:  # reference chunk k: a fresh decoder, primed from its 25 context frames
                        base = k * RC - (RX if k * RC - RX > 0 else k * RC)
                        cs, fed, emit_s, ctx_s = dec.stream(B, RX + RC), base, 0, (k * RC - base) * up
                    hi = min(avail, cend)
                    if hi > fed:
                        cc = self._stream_window(codes, pre, R, end, fed, hi)
                        cs.feed(cc)
                        fed = hi
                    n = max(cs.ns - ctx_s - emit_s, 0)
                    ended = t_end is not None and fed >= t_end
                    for b in range(B):
                        if done[b] or n == 0:
                            continue
                        lo_s = max(gpos, skip[b])
                        hi_s = gpos + n if cap[b] is None else min(gpos + n, cap[b])
                        last = cap[b] is not None and (gpos + n >= cap[b] or ended)
                        if hi_s <= lo_s and not last:
                            continue
                        o = ctx_s + emit_s + (lo_s - gpos)
                        chunk = cs.pcm[b, o:o + max(hi_s - lo_s, 0)]
                        done[b] = last
                        if unchecked:  # flags copied behind the feed that produced this PCM: the caller waits on it anyway
                            HandoffWatch(sessions).check()
                            unchecked = False
                        yield b, chunk, last
                    emit_s += n
                    gpos += n
                    if fed == cend and not ended:  # chunk k complete (its 555-sample tail is dropped): next chunk
                        cs.close()
                        cs, k = None, k + 1
                        continue
                    break
                if t_end is not None and fed >= t_end:
                    for b in range(B):  # rows whose output was complete before the last window
                        if not done[b]:
                            if unchecked:
                                HandoffWatch(sessions).check()
                                unchecked = False
                            done[b] = True
                            yield b, torch.zeros(0, device=codes.device), True
                if all(done):
                    break
        finally:
            if cs is not None:
                cs.close()
