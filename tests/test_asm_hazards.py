"""The inline-asm loads of the product kernels (attention.hip: asm_ld16 / asm_ld4 in attn_oproj_k; gemm.hip: gemv_wt's
epilogue-operand prefetch and gathered-row index load -- hipcc inserts no waits for them) are read only after the
counted `s_waitcnt vmcnt` that retires them: tools/asm_load_hazards.py scans the gfx950 assembly in layout order for
any instruction touching a destination register of a load still in flight (a register-allocator copy placed above the
wait made attn_oproj_hs_k read stale K / V / q rows in round 4: nondeterministic bf16 results).  CPU only: hipcc
cross-compiles the device code (attention.hip ~40 s, gemm.hip ~3.5 min the first time); the assembly is cached under
qwen3-tts_amd/build/asm/ by a digest of the sources and flags, so later runs only re-scan it."""
import hashlib
import os
import shutil
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "qwen3-tts_amd")
SRCS = ["attention.hip", "gemm.hip"]


def _asm(src, tmp_path):
    sys.path.insert(0, PKG)
    import build as _b
    path = os.path.join(PKG, "csrc", src)
    h = hashlib.sha256(" ".join(_b.FLAGS).encode())
    for p in [path] + _b._headers():
        with open(p, "rb") as f:
            h.update(f.read())
    cache = os.path.join(PKG, "build", "asm")
    os.makedirs(cache, exist_ok=True)
    out = os.path.join(cache, f"{src}.{h.hexdigest()[:16]}.s")
    if not os.path.exists(out):
        tmp = str(tmp_path / (src + ".s"))
        r = subprocess.run([_b.HIPCC] + _b.FLAGS + ["--cuda-device-only", "-S", path, "-o", tmp], capture_output=True,
                           text=True, timeout=900)
        assert r.returncode == 0, r.stderr
        shutil.move(tmp, out)
    with open(out) as f:
        return f.read()


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"), reason="no hipcc")
@pytest.mark.parametrize("src", SRCS)
def test_asm_loads_have_no_early_reads(src, tmp_path):
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import asm_load_hazards as hz
    asm = _asm(src, tmp_path)
    checked = 0
    for name, body in hz.functions(asm):
        if ";;#ASMSTART" not in body or "global_load" not in body:
            continue
        checked += 1
        bad = hz.check(body)
        assert not bad, f"{src} {name}: reads of in-flight asm-load registers: {bad[:5]}"
    assert checked > 0, f"{src}: no kernel with inline-asm loads found"
    print(f"\n  {src}: {checked} kernels with inline-asm loads, no early reads")
