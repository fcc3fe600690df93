"""GPU idle gaps inside one streamed first packet (1.7B synthetic, B=8, 200-token prompts): the kernel timeline of
the 5th first() call from torch.profiler, every gap > 40 us with the kernels either side and the host-side op that
was running when the GPU went idle."""
import os
import sys
import time
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "qwen3-tts_amd"))
import bench  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    from qwen_tts import Qwen3TTSModel
    B = int(os.environ.get("QT_FPG_B", "8"))
    if os.environ.get("QT_FPG_VC"):  # configs[4]: voice-clone prompt (encode + x-vector) + stream first packet
        return _profile(*_vc_first(B))
    cfg, W, CW = bench.make_weights("1.7b-customvoice", dev, 1, 0)
    tts = Qwen3TTSModel.from_pretrained("synthetic:1.7b-customvoice", device_map=str(dev), dtype=torch.bfloat16,
                                        weights=W, codec_weights=CW)
    m = tts.model
    spk = ["vivian", "ryan", "serena", "aiden", "eric", "dylan", "sohee", "ono_anna"]
    gen = dict(do_sample=True, top_k=50, top_p=1.0, temperature=0.9, subtalker_dosample=True, subtalker_top_k=50,
               subtalker_top_p=1.0, subtalker_temperature=0.9, repetition_penalty=1.05, ignore_eos=True)
    ids = [bench.synth_ids(200, i) for i in range(B)]
    kw = dict(input_ids=ids, languages=["english"] * B, speakers=spk[:B], non_streaming_mode=False, seed=7,
              max_new_tokens=257)

    def first():
        for _ in m.stream(**kw, **gen):
            break
        torch.cuda.synchronize()
    _profile(first, B)


def _vc_first(B):
    """configs[4] per GPU (tools/config_bench.py config4): B 3 s reference clips, ICL prompts, 120-token texts."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden"))
    from cases import ref_audio, ref_text_ids
    from qwen_tts import Qwen3TTSModel
    tts = Qwen3TTSModel.from_pretrained("synthetic:1.7b-base", dtype=torch.bfloat16)
    m = tts.model
    clips = [(ref_audio(72000, 100 + i), 24000) for i in range(B)]
    ids = [bench.synth_ids(120, 50 + i) for i in range(B)]
    ref_ids = [ref_text_ids(40, 60 + i) for i in range(B)]
    gen = dict(max_new_tokens=257, do_sample=True, top_k=50, top_p=1.0, temperature=0.9, subtalker_dosample=True,
               subtalker_top_k=50, subtalker_top_p=1.0, subtalker_temperature=0.9, repetition_penalty=1.05,
               ignore_eos=True)

    def first():
        items = tts.create_voice_clone_prompt(ref_audio=clips, ref_text=["ref"] * B)
        vcp = tts._prompt_items_to_voice_clone_prompt(items)
        for _ in m.stream(input_ids=ids, ref_ids=ref_ids, voice_clone_prompt=vcp, languages=["english"] * B,
                          non_streaming_mode=False, **gen):
            break
        torch.cuda.synchronize()
    return first, B


def _profile(first, B):
    for _ in range(4):
        first()
    from torch.profiler import profile, ProfilerActivity
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        t0 = time.perf_counter()
        first()
        wall = (time.perf_counter() - t0) * 1e3
    ev = [e for e in prof.events() if e.device_type == torch.autograd.DeviceType.CUDA]
    ev.sort(key=lambda e: e.time_range.start)
    cpu = [e for e in prof.events() if e.device_type == torch.autograd.DeviceType.CPU]
    t_begin = min(e.time_range.start for e in cpu)
    print(f"B={B} wall {wall:.2f} ms; {len(ev)} GPU ops, first at +{(ev[0].time_range.start - t_begin) / 1e3:.2f} ms, "
          f"last ends +{(max(e.time_range.end for e in ev) - t_begin) / 1e3:.2f} ms")
    dump = os.environ.get("QT_FPG_DUMP")
    if dump:  # every GPU op: name, stream, start / end in us from the call's start
        with open(dump, "w") as f:
            for e in ev:
                f.write(f"{(e.time_range.start - t_begin) / 1e3:.3f}\t{(e.time_range.end - t_begin) / 1e3:.3f}\t"
                        f"{getattr(e, 'device_resource_id', -1)}\t{e.name[:90]}\n")
    busy = sum(e.time_range.end - e.time_range.start for e in ev) / 1e3
    print(f"GPU busy {busy:.2f} ms")
    _top(ev)
    # the span before the first frame-graph kernel: prompt assembly + prefill
    cut = [e for e in ev if "gemv_wt" in e.name or "cp_" in e.name]
    if cut:
        pre = [e for e in ev if e.time_range.end <= cut[0].time_range.start]
        print(f"before the first GEMV: {len(pre)} ops, span {(cut[0].time_range.start - ev[0].time_range.start) / 1e3:.2f} ms")
        _top(pre, 12)
    end = ev[0].time_range.end
    for a, b in zip(ev, ev[1:]):
        end = max(end, a.time_range.end)
        gap = b.time_range.start - end
        if gap > 40:
            # innermost CPU op active at the gap start
            act = [c for c in cpu if c.time_range.start <= end <= c.time_range.end]
            act.sort(key=lambda c: c.time_range.end - c.time_range.start)
            names = " < ".join(c.name[:40] for c in act[:3])
            print(f"  gap {gap / 1e3:6.2f} ms at +{(end - t_begin) / 1e3:6.2f}: {a.name[:40]} -> {b.name[:40]} | cpu: {names}")



def _top(ev, n=20):
    agg = {}
    for e in ev:
        k = e.name[:70]
        t, c = agg.get(k, (0.0, 0))
        agg[k] = (t + (e.time_range.end - e.time_range.start) / 1e3, c + 1)
    for k, (t, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:n]:
        print(f"  {t:7.3f} ms {c:5d}x  {k}")


if __name__ == "__main__":
    main()
