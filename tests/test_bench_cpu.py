"""bench.py's multi-rank launcher on host CPUs (gloo): `--gpus 2` without a torchrun environment starts
2 ranks itself, the world size comes from the process group, and rank 0 prints one JSON line."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*extra):
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu", "--steps", "3",
                        "--warmup", "1", *extra], capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


def test_bench_launcher_spawns_two_gloo_ranks():
    out = _run("--gpus", "2")
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2"
    assert out["steps"] == 3 and out["value"] > 0 and out["ms_per_step"] > 0


def test_bench_single_rank_default():
    out = _run()
    assert out["n_gpus"] == 1


def test_bench_rejects_world_size_mismatch():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu", "--gpus", "2"],
                       capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert p.returncode != 0 and "WORLD_SIZE" in p.stderr
