"""bench.py's multi-GPU launch on CPU (QT_BENCH_DRYRUN=1: the launcher, rank init, barriers, max/sum reductions and the
JSON line, with no model and no GPU).  `bench.py --gpus N` must run N ranks by itself when no torch.distributed
launcher is around it (the driver's 1 -> 8 scaling run), and refuse a WORLD_SIZE that differs from --gpus."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT", "QT_BENCH_LAUNCHER")}
    env.update(QT_BENCH_DRYRUN="1", OMP_NUM_THREADS="1", **kw)
    return env


def _json_line(out: str):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [2, 3])
def test_bench_gpus_n_launches_n_ranks(n):
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(n), "--steps", "3",
                        "--warmup", "1"], env=_env(), cwd=REPO, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    j = _json_line(r.stdout)
    assert j["n_gpus"] == n
    assert j["launcher"] == "self"
    assert j["dist_backend"] == "gloo"
    assert len(j["per_rank_value"]) == n
    # whole-job value = summed audio / max wall time: every rank did the same work, so about n x one rank's rate
    assert j["audio_seconds"] == pytest.approx(n * 3 * 8 * 256 * 1920 / 24000.0)
    assert j["value"] <= sum(j["per_rank_value"]) * 1.0001
    assert j["value"] >= 0.7 * sum(j["per_rank_value"])


def test_bench_single_gpu_needs_no_launcher():
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "2", "--warmup", "0"],
                       env=_env(), cwd=REPO, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    j = _json_line(r.stdout)
    assert j["n_gpus"] == 1 and j["launcher"] is None and len(j["per_rank_value"]) == 1


def test_bench_refuses_world_size_mismatch():
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "4", "--steps", "1"],
                       env=_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"), cwd=REPO, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode != 0
    assert "WORLD_SIZE=1" in (r.stderr + r.stdout)
