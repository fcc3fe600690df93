"""Build libqwen3tts_amd.so (all HIP kernels + the C ABI of include/qwen3tts_amd.h) for gfx950.

    python qwen3-tts_amd/build.py [--jobs N] [--force]

Plain hipcc, one object per .hip source (parallel), linked into lib/libqwen3tts_amd.so in-tree so the
library travels with the repo snapshot to the GPU box.  Staleness is decided by content, not mtime: every
object records the digest of its source + the shared headers + the flags, and the library carries the digest
of the whole source set as `qt_build_id()` (a generated one-line source), which `qwen_tts._hip` compares with
the sources next to it at load time -- a library that does not match the tree it ships with is refused.
"""
import argparse
import concurrent.futures as cf
import glob
import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(HERE, "build")
LIB = os.path.join(HERE, "lib", "libqwen3tts_amd.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wno-pass-failed", "-munsafe-fp-atomics"]
# probe build (--probe): the A/B tools' measurement knobs (getenv) and phase early exits compiled in, linked as a
# separate library that tools select with QWEN3TTS_AMD_LIB; the product library never reads the environment
PROBE_FLAGS = FLAGS + ["-DQT_PROBE_BUILD"]
PROBE_BUILD = os.path.join(HERE, "build_probe")
PROBE_LIB = os.path.join(HERE, "lib", "libqwen3tts_amd_probe.so")


def _read(p):
    with open(p, "rb") as f:
        return f.read()


def _headers():
    return sorted(glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(HERE, "..", "include", "*.h")))


def _sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def source_digest(csrc=CSRC, probe=False) -> str:
    """sha256 over every kernel source, the shared headers and the compile flags (16 hex digits)."""
    h = hashlib.sha256(" ".join(PROBE_FLAGS if probe else FLAGS).encode())
    inc = os.path.join(os.path.dirname(csrc), "..", "include")
    files = sorted(glob.glob(os.path.join(csrc, "*.hip")) + glob.glob(os.path.join(csrc, "*.h"))
                   + glob.glob(os.path.join(inc, "*.h")))
    for p in files:
        h.update(os.path.basename(p).encode())
        h.update(_read(p))
    return h.hexdigest()[:16]


def _obj_digest(src, flags):
    h = hashlib.sha256(" ".join(flags).encode())
    for p in [src] + _headers():
        h.update(_read(p))
    return h.hexdigest()


def _compile(src, force=False, probe=False):
    flags = PROBE_FLAGS if probe else FLAGS
    obj = os.path.join(PROBE_BUILD if probe else BUILD, os.path.basename(src) + ".o")
    stamp = obj + ".sha"
    dig = _obj_digest(src, flags)
    if not force and os.path.exists(obj) and os.path.exists(stamp) and _read(stamp).decode() == dig:
        return obj
    cmd = [HIPCC] + flags + ["-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
    with open(stamp, "w") as f:
        f.write(dig)
    return obj


def _build_id_obj(bid, probe=False):
    src = os.path.join(PROBE_BUILD if probe else BUILD, "build_id.hip")
    with open(src, "w") as f:
        f.write(f'extern "C" const char* qt_build_id() {{ return "{bid}"; }}\n')
    return _compile(src, probe=probe)


def build(jobs=8, verbose=True, force=False, probe=False):
    bdir, LIB = (PROBE_BUILD, PROBE_LIB) if probe else (BUILD, globals()["LIB"])
    os.makedirs(bdir, exist_ok=True)
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    srcs = _sources()
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, force, probe), srcs))
    bid = source_digest(probe=probe) + ("-probe" if probe else "")
    objs.append(_build_id_obj(bid, probe))
    stamp = LIB + ".sha"
    link_key = bid + " " + " ".join(sorted(os.path.basename(o) for o in objs))
    if force or not os.path.exists(LIB) or not os.path.exists(stamp) or _read(stamp).decode() != link_key:
        cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", LIB] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr}")
        with open(stamp, "w") as f:
            f.write(link_key)
    if verbose:
        print(f"built {LIB} (build id {bid})")
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=8)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--probe", action="store_true", help="measurement build: lib/libqwen3tts_amd_probe.so")
    a = ap.parse_args()
    sys.exit(0 if build(a.jobs, force=a.force, probe=a.probe) else 1)
