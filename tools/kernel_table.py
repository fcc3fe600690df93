"""The bench's per-kernel decode table (bench.decode_kernel_table: every decode kernel of a frame at its production
shape, 1.7B CustomVoice, B = 8, bf16) without the bench's timed steps: one short generate creates the sessions, then
the table.  For A/B sweeps of the library's GEMV knobs (QT_GEMV_*), one process per setting."""
import os
import sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "qwen3-tts_amd"))
import bench  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    from qwen_tts import Qwen3TTSModel
    B = 8
    cfg, W, CW = bench.make_weights("1.7b-customvoice", dev, 1, 0)
    tts = Qwen3TTSModel.from_pretrained("synthetic:1.7b-customvoice", device_map=str(dev), dtype=torch.bfloat16,
                                        weights=W, codec_weights=CW)
    spk = ["vivian", "ryan", "serena", "aiden", "eric", "dylan", "sohee", "ono_anna"]
    ids = [bench.synth_ids(200, i) for i in range(B)]
    tts.model.generate(input_ids=ids, languages=["english"] * B, speakers=spk, non_streaming_mode=False, seed=1,
                       max_new_tokens=4, do_sample=True, top_k=50, ignore_eos=True)
    tab = bench.decode_kernel_table(tts, B, 330)
    tag = os.environ.get("KT_TAG", "default")
    print(tag, " ".join(f"{e['name']}={e['avg_us']:.2f}" for e in tab), flush=True)


if __name__ == "__main__":
    main()
