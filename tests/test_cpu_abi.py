"""CPU-only: the C-ABI library loads and exports every symbol declared in include/qwen3tts_amd.h."""
import os
import re

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_declared_symbol():
    from qwen_tts import _hip
    L = _hip.load_library()
    hdr = open(os.path.join(REPO, "include", "qwen3tts_amd.h")).read()
    declared = set(re.findall(r"\b(?:int|long long) (qt_\w+)\(", hdr))
    assert declared == set(_hip.EXPORTS)
    for name in declared:
        assert hasattr(L, name), name
