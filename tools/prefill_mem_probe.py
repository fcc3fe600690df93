"""Where does device memory go per new prompt length?  Tiny model, 12 distinct prompt lengths x 2 uses each, twice
over; prints torch.cuda.memory_allocated after each length and the live CUDAGraph count (QT_PREFILL_GRAPH=0 to A/B
the captured prefill graphs)."""
import gc
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "qwen3-tts_amd"), os.path.join(REPO, "tests", "golden")):
    sys.path.insert(0, p)

import torch  # noqa: E402

from cases import gen_kwargs, make_inputs, talker_cases  # noqa: E402
from oracle import load_preset, synth_state_dict, talker_param_specs  # noqa: E402
from qwen_tts.model import TTSModel  # noqa: E402

cfg, _ = load_preset("tiny-customvoice")
W = {k: torch.from_numpy(v) for k, v in synth_state_dict(talker_param_specs(cfg)).items()}
m = TTSModel(cfg, W, dtype="fp32")
case = dict(talker_cases()["cv_b1_nonstream"], max_new_tokens=6)
prev = None
for rep in range(3):
    for n in range(3, 15):
        c = dict(case, texts=[n])
        ids, ins, vcp, ref_ids = make_inputs(c, 0, cfg["talker_config"]["hidden_size"])
        for _ in range(2):
            m.generate(input_ids=ids, languages=c["languages"], speakers=c["speakers"],
                       non_streaming_mode=c["non_streaming_mode"], **gen_kwargs(c))
        torch.cuda.synchronize()
        gc.collect()
        mem = torch.cuda.memory_allocated()
        graphs = sum(1 for o in gc.get_objects() if isinstance(o, torch.cuda.CUDAGraph))
        lens = [len(s.prefill) for s in m.engine.all_sessions()]
        print(f"rep {rep} P-text {n}: allocated {mem} (+{0 if prev is None else mem - prev}) graphs {graphs} "
              f"prefill entries {lens}", flush=True)
        prev = mem
