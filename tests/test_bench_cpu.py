"""bench.py's launch contract on the CPU (no GPU work): `--gpus N` means N ranks.

`python bench.py --gpus 2` with no launcher starts torch.distributed.run with two ranks as a child process, and the
rank-0 line says n_gpus 2; `--gpus N` that disagrees with an existing WORLD_SIZE is an error, not a world-1 line.
`--dry-run` stops each rank after the process group has formed (gloo here), so no GPU is needed.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                              "MASTER_PORT")}
    env.update(HLGS_DIST_BACKEND="gloo", OMP_NUM_THREADS="1", **kw)
    return env


def _line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def test_gpus_2_without_launcher_starts_two_ranks():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run"], env=_env(), capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = _line(r.stdout)
    assert line["n_gpus"] == 2 and line["ranks_joined"] == 2 and line["gpus_arg"] == 2


def test_gpus_1_default_is_one_rank():
    r = subprocess.run([sys.executable, BENCH, "--dry-run"], env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert _line(r.stdout)["n_gpus"] == 1


def test_gpus_disagreeing_with_world_size_fails():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "8", "--dry-run"], env=_env(WORLD_SIZE="1"),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "WORLD_SIZE=1" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_gpus_zero_rejected():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "0", "--dry-run"], env=_env(), capture_output=True,
                       text=True, timeout=300)
    assert r.returncode != 0
