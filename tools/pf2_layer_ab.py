"""Prefill linears of the 1.7B talker (28 layers, distinct weights, in a HIP graph) at M rows, as bench.py's
prefill_mfma measures them: per-layer us and TFLOP/s.  With the probe library (QWEN3TTS_AMD_LIB=.../_probe.so),
QT_PF2_PP=0 leaves the ping-pong tile configurations out of gemm_pf2.hip's picker (A/B in separate processes).

    python tools/pf2_layer_ab.py [M ...]
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "qwen3-tts_amd"))
import bench  # noqa: E402
from qwen_tts import Qwen3TTSModel  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    cfg, W, CW = bench.make_weights("1.7b-customvoice", dev, 1, 0)
    tts = Qwen3TTSModel.from_pretrained("synthetic:1.7b-customvoice", device_map=str(dev), dtype=torch.bfloat16,
                                        weights=W, codec_weights=CW)
    del W, CW
    for M in [int(x) for x in sys.argv[1:]] or [680]:
        r = bench.prefill_mfma(tts, M=M, reps=5)
        print(json.dumps({"M": M, "pp": os.environ.get("QT_PF2_PP", "1"), "us_per_layer": round(r["us_per_layer"], 1),
                          "tflops": round(r["tflops"], 1)}), flush=True)


if __name__ == "__main__":
    main()
