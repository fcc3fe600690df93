"""Kernel mix of one incremental codec feed (the stream's first window: 3 frames) at the 1.7B dims, B=8, replayed
from its captured graph -- run under rocprofv3 --kernel-trace. QT_CF_N frames (default 2 = the stream's first
packet since it emits without a lookahead frame), QT_CF_B rows."""
import os
import sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "qwen3-tts_amd"))
import bench  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    from qwen_tts.codec import CodecDecoder
    from qwen_tts.weights import codec_specs, read_json, resolve_path, synthetic
    d = resolve_path("synthetic:1.7b-customvoice")
    ccfg = read_json(os.path.join(d, "speech_tokenizer", "config.json"))
    dec = CodecDecoder(ccfg, synthetic(codec_specs(ccfg), dev), dtype="bf16", device=str(dev))
    B = int(os.environ.get("QT_CF_B", "8"))
    n = int(os.environ.get("QT_CF_N", "2"))
    codes = torch.randint(1, 2048, (B, n, 16), device=dev, dtype=torch.int32)
    for _ in range(20):
        cs = dec.stream(B, 325)
        cs.feed(codes)
        cs.close()
    torch.cuda.synchronize()
    import time
    ts = []
    for _ in range(10):
        cs = dec.stream(B, 325)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        cs.feed(codes)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
        cs.close()
    ts.sort()
    print(f"B={B} first-window feed ({n} frames, replayed graph): {ts[5]:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
