"""`python bench.py --gpus N` with no launcher starts its N ranks itself (torchrun as a child
of a parent that never touches the GPU; the reference launches its ranks with mp.spawn,
perseus/detector/train.py:371-375) and every rank checks the process group's size.  Run
here on CPU through --launcher-check: the ranks join a gloo group instead of RCCL."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args, env=None):
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                          timeout=300, env=env, cwd=ROOT)


def test_two_ranks_join_without_a_launcher():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = _run("--gpus", "2", "--launcher-check", env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["world_env"] == 2
    assert line["ranks_mask"] == 0b11  # rank 0 and rank 1 both reached the all-reduce


def test_world_size_mismatch_exits_nonzero():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = _run("--gpus", "2", "--launcher-check", env=env)
    assert r.returncode != 0 and "--gpus 2" in r.stderr
