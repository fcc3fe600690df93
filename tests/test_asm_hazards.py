"""The inline-asm loads of attention.hip (asm_ld16 / asm_ld4: hipcc inserts no waits for them) are read only after
the counted `s_waitcnt vmcnt` that retires them: tools/asm_load_hazards.py scans the gfx950 assembly in layout order
for any instruction touching a destination register of a load still in flight (a register-allocator copy placed
above the wait made attn_oproj_hs_k read stale K / V / q rows: nondeterministic bf16 results).  CPU only (hipcc
cross-compiles, ~40 s); gemm.hip's asm prefetches were checked the same way (0 hazards, a 3.5 min compile)."""
import os
import shutil
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "qwen3-tts_amd")


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"), reason="no hipcc")
def test_attention_asm_loads_have_no_early_reads(tmp_path):
    sys.path.insert(0, PKG)
    import build as _b
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import asm_load_hazards as hz
    out = tmp_path / "attention.s"
    r = subprocess.run([_b.HIPCC] + _b.FLAGS + ["--cuda-device-only", "-S", os.path.join(PKG, "csrc", "attention.hip"),
                                                 "-o", str(out)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr
    asm = out.read_text()
    checked = 0
    for name, body in hz.functions(asm):
        if ";;#ASMSTART" not in body or "global_load" not in body:
            continue
        checked += 1
        bad = hz.check(body)
        assert not bad, f"{name}: reads of in-flight asm-load registers: {bad[:5]}"
    assert checked > 0
