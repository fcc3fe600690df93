"""Host-side scheduling logic that needs no GPU: the streaming codec's per-row decode windows (voice-clone reference
prefixes + generated codes + zero padding, qwen_tts.model.TTSModel._stream_window) and the data-parallel shard
assignment."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "qwen3-tts_amd"))


def _seq(pre, gen, end):
    """Row sequence as the wrapper decodes it: cat(ref_code, codes[:end]) (W:263-265)."""
    g = gen[:end] if end is not None else gen
    return g if pre is None else torch.cat([pre, g], 0)


def test_stream_window_matches_concatenated_sequences():
    from qwen_tts.model import TTSModel
    g = torch.Generator().manual_seed(3)
    B, frames = 3, 20
    codes = torch.randint(1, 2048, (B, frames + 1, 16), generator=g, dtype=torch.int32)
    pre = [torch.randint(1, 2048, (7, 16), generator=g, dtype=torch.int32), None,
           torch.randint(1, 2048, (4, 16), generator=g, dtype=torch.int32)]
    R = [7, 0, 4]
    end = [None, 12, 5]  # row 0 still running, rows 1 / 2 ended after 12 / 5 generated frames
    full = []
    for b in range(B):
        s = _seq(pre[b], codes[b], end[b] if end[b] is not None else frames)
        full.append(torch.cat([s, torch.zeros(40, 16, dtype=torch.int32)], 0))  # batch zero padding
    avail = R[0] + frames  # the running row bounds the positions known for every row
    for lo, hi in [(0, 3), (3, 11), (11, avail), (0, avail)]:
        cc = TTSModel._stream_window(codes, pre, R, end, lo, hi)
        assert cc.shape == (B, hi - lo, 16)
        for b in range(B):
            assert torch.equal(cc[b], full[b][lo:hi]), (b, lo, hi)


def test_stream_window_without_prefix_zero_pads_ended_rows():
    from qwen_tts.model import TTSModel
    codes = torch.arange(2 * 9 * 16, dtype=torch.int32).view(2, 9, 16) + 1
    cc = TTSModel._stream_window(codes, [None, None], [0, 0], [None, 4], 2, 8)
    assert torch.equal(cc[0], codes[0, 2:8])
    assert torch.equal(cc[1, :2], codes[1, 2:4]) and int(cc[1, 2:].abs().sum()) == 0


def test_shard_longest_first_balances_frames():
    from qwen_tts.dp import shard_longest_first
    lengths = [320, 64, 200, 180, 96, 310, 150, 75, 260, 128, 90, 240]
    shards = shard_longest_first(lengths, 4)
    assert sorted(i for s in shards for i in s) == list(range(len(lengths)))
    loads = [sum(lengths[i] for i in s) for s in shards]
    assert max(loads) - min(loads) <= max(lengths)


def test_bench_module_helpers():
    """bench.py imports on CPU and its pure helpers compute: algorithmic bytes of a 1.7B frame."""
    import importlib
    import json
    import os
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, repo)
    bench = importlib.import_module("bench")
    for name in ("decode_kernel_table", "attn_oproj_entry", "_gemv_entry", "_graph_us", "_pmc_traffic",
                 "whole_frame_roofline", "prefill_mfma", "attention_roofline", "cpu_baseline", "main", "main_vd64"):
        assert callable(getattr(bench, name)), name
    cfg = json.load(open(os.path.join(repo, "qwen3-tts_amd", "qwen_tts", "configs", "1.7b-customvoice", "config.json")))
    b = bench.frame_bytes(cfg, 8, 200)
    assert 5.0e9 < b < 6.0e9  # ~2.8 GB of talker weights + 15 code-predictor passes + K/V
