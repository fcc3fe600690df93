"""Benchmark: Qwen3-TTS-12Hz-1.7B CustomVoice, batch 8 x 200-token prompts, streaming-text decode
(BASELINE.json configs[2]) on the MI355X HIP path.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

One step = prefill + 256 AR frames (talker + 15-step code predictor per frame, HIP-graph replay) +
12 Hz codec decode of all 8 utterances to 24 kHz PCM.  Weak scaling: every rank serves its own batch of
8 independent utterances (data parallel, no collective on the data path; RCCL only broadcasts the
weights at init).  Weights are seeded synthetic at the ASSUMED 1.7B dims (no checkpoint offline).
value = sum over ranks of generated audio seconds / max-over-ranks wall time of the K timed steps.
Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "qwen3-tts_amd"))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def synth_ids(n, seed):
    g = np.random.default_rng([1234, seed])
    body = g.integers(1000, 150000, n).tolist()
    return torch.tensor([[151644, 77091, 198] + body + [151645, 198, 151644, 77091, 198]], dtype=torch.long)


def make_weights(preset, dev, world, rank):
    from qwen_tts.weights import codec_specs, read_json, resolve_path, synthetic, talker_specs
    d = resolve_path(f"synthetic:{preset}")
    cfg = read_json(os.path.join(d, "config.json"))
    ccfg = read_json(os.path.join(d, "speech_tokenizer", "config.json"))
    specs_t, specs_c = talker_specs(cfg), codec_specs(ccfg)
    if world > 1:  # rank 0 generates, RCCL broadcast over xGMI (the only collective of the design)
        from qwen_tts.dp import broadcast_weights
        W = synthetic(specs_t, dev) if rank == 0 else {n: torch.empty(s, device=dev) for n, s in specs_t}
        CW = synthetic(specs_c, dev) if rank == 0 else {n: torch.empty(s, device=dev) for n, s in specs_c}
        broadcast_weights(W)
        broadcast_weights(CW)
    else:
        W, CW = synthetic(specs_t, dev), synthetic(specs_c, dev)
    return cfg, W, CW


ROOF_KERNEL = "gemv_wt<bf16,bf16,bf16,WPB=4,U=4,rms,fold=2> (talker MLP gate-up decode GEMV, N=12288 K=2048 M=8)"


def gateup_bytes(eng, B):
    """Algorithmic HBM bytes of one talker gate-up launch: bf16 weight tiles + A rows (the bf16 residual shadow in
    bf16 mode) + bf16 SwiGLU out."""
    t = eng.talker
    L = t.layers[0].gu
    a_bytes = 2 if eng.wdt == torch.bfloat16 else 4
    return L.w.numel() * L.w.element_size() + B * t.H * a_bytes + B * t.I * L.w.element_size()


def kernel_roofline(tts, B, reps=10):
    """Dominant decode kernel timed live: a HIP graph of the 28 production gate-up launches (one per layer,
    distinct weights, so every launch streams HBM as in a frame), replayed `reps` times between HIP events
    recorded on the capture stream.  Per-launch time includes the in-graph dispatch gap (conservative)."""
    from qwen_tts import _hip, kernels as Kn
    eng = tts.model.engine
    t = eng.talker
    dev = eng.dev
    x = torch.randn(B, t.H, device=dev).to(eng.wdt)  # production A: the bf16 residual shadow (fp32 in fp32 mode)
    h = torch.empty(B, t.I, dtype=eng.wdt, device=dev)

    def run():
        for L in t.layers:
            Kn.gemm(x, L.gu, h, B, t.H, t.I, rms=True, eps=t.eps, epi=_hip.EPI_SWIGLU)
    st = torch.cuda.Stream(device=dev)
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        run()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=st):
            run()
        g.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            g.replay()
        e1.record(st)
    torch.cuda.synchronize()
    n = reps * len(t.layers)
    us = e0.elapsed_time(e1) * 1e3 / n
    byt = gateup_bytes(eng, B)
    return dict(avg_us=us, bytes=byt, gbs=byt / (us * 1e-6) / 1e9, launches=n)


def attention_roofline(tts, B, L, reps=10):
    """North-star secondary roofline: the talker decode attention (q/k norm + RoPE + KV append + GQA attention,
    attn_decode_k) at cache length L, 28 launches over distinct per-layer caches (as in a frame) in a HIP graph.
    Algorithmic bytes per launch = the K and V rows read: B x Hkv x L x D x 2 x sizeof(bf16)."""
    from qwen_tts import kernels as Kn
    eng = tts.model.engine
    t = eng.talker
    dev = eng.dev
    nl = len(t.layers)
    kc = [torch.randn(B, t.Hkv, L + 1, t.D, device=dev).to(eng.kv_dtype) for _ in range(nl)]
    vc = [torch.randn(B, t.Hkv, L + 1, t.D, device=dev).to(eng.kv_dtype) for _ in range(nl)]
    qkv = torch.randn(B, (t.Hq + 2 * t.Hkv) * t.D, device=dev)
    att = torch.empty(B, t.Hq * t.D, dtype=eng.wdt, device=dev)
    pos = torch.full((B,), L - 1, dtype=torch.int32, device=dev)
    rb = torch.arange(B, dtype=torch.int32, device=dev)
    zero = torch.zeros(B, dtype=torch.int32, device=dev)
    t.ensure_rope(L + 4, dev)
    L0 = t.layers[0]

    def run():
        for i in range(nl):
            Kn.decode_attention(qkv, B, t.Hq, t.Hkv, t.D, L0.q_norm, L0.k_norm, t.eps, t.cos, t.sin, pos, rb, pos,
                                zero, kc[i], vc[i], L + 1, att)
    st = torch.cuda.Stream(device=dev)
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        run()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=st):
            run()
        g.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            g.replay()
        e1.record(st)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / (reps * nl)
    byt = B * t.Hkv * L * t.D * 2 * kc[0].element_size()
    return dict(avg_us=us, bytes=byt, gbs=byt / (us * 1e-6) / 1e9, keys=L)


def cpu_baseline(B, prompt, frames, threads):
    """Oracle (CPU fp32 restatement of the reference) on a bounded sample of the same workload."""
    from oracle import CodecOracle, TalkerOracle, build_prompts, codec_param_specs, generate, load_preset
    from oracle.talker import talker_param_specs
    torch.set_num_threads(threads)
    cfg, ccfg = load_preset("1.7b-customvoice")
    g = torch.Generator().manual_seed(0)
    W = {n: 0.02 * torch.randn(s, generator=g) for n, s in talker_param_specs(cfg)}
    CW = {n: 0.02 * torch.randn(s, generator=g) for n, s in codec_param_specs(ccfg)}
    o, co = TalkerOracle(cfg, W), CodecOracle(ccfg, CW)
    ids = [synth_ids(prompt, i) for i in range(B)]
    spk = ["vivian", "ryan", "serena", "aiden", "eric", "dylan", "sohee", "ono_anna"][:B]
    t0 = time.time()
    with torch.no_grad():
        emb, mask, trail, pad = build_prompts(o, ids, ["english"] * B, (spk * 8)[:B], None, False)
        res = generate(o, emb, mask, trail, pad, max_new_tokens=frames + 1, do_sample=True, ignore_eos=True)
        codes = torch.stack(res.codes)
        wav = co.decode(codes)
    dt = time.time() - t0
    audio = sum(w.shape[0] for w in wav) / 24000.0
    return dict(value=audio / dt, unit="audio-seconds/sec", cores=threads, kind="port",
                sample=f"oracle fp32, 1.7B dims, B={B} x {prompt}-token prompts, {frames} frames + codec, {dt:.1f}s")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--frames", type=int, default=256)
    ap.add_argument("--prompt-tokens", type=int, default=200)
    ap.add_argument("--preset", default="1.7b-customvoice")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--cpu-baseline", type=int, default=1)
    ap.add_argument("--cpu-frames", type=int, default=24)
    ap.add_argument("--roofline", type=int, default=1)
    ap.add_argument("--row-groups", type=int, default=1,
                    help="decode the per-GPU batch as this many concurrent row groups (streams)")
    a = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # test-only overrides: rehearse the N>1 path on one GPU (all ranks on cuda:0, gloo collectives)
    backend = os.environ.get("QT_BENCH_BACKEND", "nccl")  # nccl == RCCL over xGMI on ROCm
    if os.environ.get("QT_BENCH_SAME_DEVICE") == "1":
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device(f"cuda:{local}")
    dist = None
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    from qwen_tts import Qwen3TTSModel
    cfg, W, CW = make_weights(a.preset, dev, world, rank)
    tts = Qwen3TTSModel.from_pretrained(f"synthetic:{a.preset}", device_map=str(dev),
                                        dtype=torch.bfloat16 if a.dtype == "bf16" else torch.float32,
                                        weights=W, codec_weights=CW)
    del W, CW
    torch.cuda.empty_cache()
    tts.model.engine.row_groups = a.row_groups
    B = a.batch
    ids = [synth_ids(a.prompt_tokens, rank * 1000 + i) for i in range(B)]
    spk = (["vivian", "ryan", "serena", "aiden", "eric", "dylan", "sohee", "ono_anna"] * 8)[:B]
    langs = ["english"] * B
    gen = dict(max_new_tokens=a.frames + 1, do_sample=True, top_k=50, top_p=1.0, temperature=0.9,
               subtalker_dosample=True, subtalker_top_k=50, subtalker_top_p=1.0, subtalker_temperature=0.9,
               repetition_penalty=1.05, ignore_eos=True)

    def step(seed):
        t0 = time.perf_counter()
        codes, _ = tts.model.generate(input_ids=ids, languages=langs, speakers=spk, non_streaming_mode=False,
                                      seed=seed, **gen)
        wavs, sr = tts.model.speech_tokenizer.decode([{"audio_codes": c} for c in codes])
        return sum(w.shape[0] for w in wavs) / sr, time.perf_counter() - t0

    for i in range(a.warmup):
        step(100 + i)

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    barrier()
    t0 = time.perf_counter()
    audio, lat = 0.0, []
    for i in range(a.steps):
        s_audio, s_t = step(i)
        audio += s_audio
        lat.append(s_t)
    barrier()
    dt = time.perf_counter() - t0
    if dist is not None:
        from qwen_tts.dp import reduce_timing
        dt, audio = reduce_timing(dt, audio, device=dev)
    value = audio / dt
    # talker cache length at the end of a timed step (prompt + frames), before stream() reuses the sessions
    L_end = max(int(ss.meta["kv_pos"].max().item()) for ss in tts.model.engine.all_sessions())
    # first packet (SURVEY §8 metric): request submit -> first PCM chunk delivered by stream(), p50 of 3 after a
    # warmup, on this rank's batch of B and on a single utterance
    def first_packet(n):
        t0 = time.perf_counter()
        for _ in tts.model.stream(input_ids=ids[:n], languages=langs[:n], speakers=spk[:n], non_streaming_mode=False,
                                  seed=7, **gen):
            break
        torch.cuda.synchronize()
        return time.perf_counter() - t0
    fp = {}
    for n in (B, 1):
        first_packet(n)
        fp[n] = 1e3 * float(np.median([first_packet(n) for _ in range(3)]))
    roof = attn_roof = None
    if a.roofline and rank == 0:
        r = kernel_roofline(tts, B)
        traffic = None
        pmcs = sorted(f for f in os.listdir(os.path.join(REPO, "profiles")) if f.endswith("_pmc_gateup.json"))
        if pmcs:  # the newest round's PMC traffic of this kernel (tools/pmc_gateup.py + tools/pmc_reduce.py)
            traffic = json.load(open(os.path.join(REPO, "profiles", pmcs[-1]))).get("hbm_bytes_per_launch")
        roof = {"bound": "hbm", "kernel": ROOF_KERNEL, "achieved": round(r["gbs"], 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(r["gbs"] / HBM_PEAK_GBS, 4), "traffic": traffic,
                "avg_launch_us": round(r["avg_us"], 2), "bytes_per_launch": int(r["bytes"]),
                "timed_launches": r["launches"]}
        # decode attention at the run's mean cache length (prompt + half the frames)
        L_mean = max(L_end - a.frames // 2, 1)
        ra = attention_roofline(tts, B, L_mean)
        attn_roof = {"bound": "hbm", "kernel": f"attn_decode_k (talker decode attention, B={B}, {L_mean} keys)",
                     "achieved": round(ra["gbs"], 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(ra["gbs"] / HBM_PEAK_GBS, 4), "avg_launch_us": round(ra["avg_us"], 2),
                     "bytes_per_launch": int(ra["bytes"])}
    cpu = None
    if a.cpu_baseline and rank == 0 and world == 1:
        cpu = cpu_baseline(B, a.prompt_tokens, a.cpu_frames, int(os.environ.get("OMP_NUM_THREADS", "16")))
    if rank == 0:
        per_utt_rtf = value / (B * world)
        out = {"metric": "audio-seconds/sec (RTF) + p50 first-packet latency, 1.7B @ batch 1/8, 1->8 GPU",
               "value": round(value, 3), "unit": "audio-seconds/sec", "n_gpus": world, "steps": a.steps,
               "warmup": a.warmup, "ms_per_step": round(1e3 * dt / a.steps, 2), "higher_is_better": True,
               "scaling": "weak", "vs_baseline": None, "dtype": a.dtype, "data": "synthetic (seeded weights + token ids)",
               "config": {"workload": f"Qwen3-TTS-12Hz-{a.preset} B={B}/GPU x {a.prompt_tokens}-token prompts, "
                                      f"streaming text, {a.frames} frames + codec decode",
                          "global_batch": B * world, "seq_len": a.prompt_tokens, "frames": a.frames,
                          "parallelism": f"dp{world}"},
               "rtf_per_utterance": round(per_utt_rtf, 2),
               "first_packet_p50_ms": round(fp[B], 1), "first_packet_p50_ms_b1": round(fp[1], 1),
               "full_batch_latency_p50_ms": round(1e3 * float(np.median(lat)), 1),
               "roofline": roof, "decode_attention_roofline": attn_roof, "cpu_baseline": cpu}
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
