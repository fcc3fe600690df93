"""The inline-asm loads of the product kernels (attention.hip: asm_ld16 / asm_ld4 in attn_oproj_k; gemm.hip: gemv_wt's
epilogue-operand prefetch and gathered-row index load -- hipcc inserts no waits for them) are read only after the
counted `s_waitcnt vmcnt` that retires them: tools/asm_load_hazards.py scans the gfx950 assembly in layout order for
any instruction touching a destination register of a load still in flight (a register-allocator copy placed above the
wait made attn_oproj_hs_k read stale K / V / q rows in round 4: nondeterministic bf16 results).  CPU only: hipcc
cross-compiles the device code (attention.hip ~40 s, gemm.hip ~3.5 min the first time); the assembly is cached under
qwen3-tts_amd/build/asm/ by a digest of the sources and flags, so later runs only re-scan it.

The persistent engines are checked for their own hand-written ordering: talker_tail.hip's loader waves publish a ring
slot behind an asm `s_waitcnt vmcnt(16)` that is right only if exactly the slot's 16 LDS-DMA transfers are the VMEM ops
in flight before it (tools/asm_load_hazards.py check_ring); in both engines every sc1 flag store follows an
`s_waitcnt vmcnt(0)` after the sc1 payload stores it publishes (check_r1: the R1 hand-off order)."""
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


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"), reason="no hipcc")
@pytest.mark.parametrize("src,kernel,ring_waits", [("talker_tail.hip", "talker_tail_k", 1),
                                                    ("cp_engine.hip", "cp_step_k", 0)])
def test_engine_ring_counts_and_r1_order(src, kernel, ring_waits, tmp_path):
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import asm_load_hazards as hz
    asm = _asm(src, tmp_path)
    n_fn = 0
    for name, body in hz.functions(asm):
        if kernel not in name:
            continue
        n_fn += 1
        bad, seen = hz.check_ring(body)
        assert not bad, f"{src} {name}: ring slot waits not matching their LDS-DMA run: {bad[:3]}"
        assert len(seen) == ring_waits, (name, len(seen))
        bad, nflags = hz.check_r1(body)
        assert not bad, f"{src} {name}: sc1 flag stores before the payload drain: {bad[:3]}"
        assert nflags >= 3, (name, nflags)
    assert n_fn > 0
    print(f"\n  {src}: {n_fn} kernel(s), ring waits and R1 flag order clean")


def test_checkers_catch_mutations():
    """The engine checks themselves, on hand-written bodies: a slot wait after 15 transfers or after a foreign VMEM op,
    and a flag store with an sc1 payload store not drained, are reported; the correct forms are not."""
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import asm_load_hazards as hz
    dma = "\n".join([";;#ASMSTART", "global_load_lds_dwordx4 v[2:3], off nt", ";;#ASMEND"])
    wait = "\n".join([";;#ASMSTART", "s_waitcnt vmcnt(16)", ";;#ASMEND"])
    ok = "\n".join([dma] * 16 + [wait])
    assert hz.check_ring(ok) == ([], [len(ok.split(chr(10))) - 2])
    assert hz.check_ring("\n".join([dma] * 15 + [wait]))[0]
    assert hz.check_ring("\n".join([dma] * 16 + ["global_load_dword v1, v[2:3], off"] + [wait]))[0]
    pub = ["buffer_store_dword v1, v2, s[0:3], 0 offen sc1", "s_waitcnt vmcnt(0)",
           "global_store_dword v0, v3, s[4:5] offset:16 sc1"]
    assert hz.check_r1("\n".join(pub)) == ([], 1)
    assert hz.check_r1("\n".join([pub[0], pub[2]]))[0]
