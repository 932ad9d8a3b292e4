"""bench.py's launcher checks, which run before any GPU is touched: a
launcher's WORLD_SIZE that contradicts --gpus, and --stub outside config 4,
fail loudly instead of timing something else."""
import os
import subprocess
import sys

from conftest import ROOT


def _run(args, **env):
    e = dict(os.environ, **env)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          timeout=300, cwd=ROOT, env=e)


def test_world_size_must_match_gpus():
    r = _run(["--gpus", "3"], WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr


def test_stub_needs_config4():
    r = _run(["--stub", "--config", "3"])
    assert r.returncode != 0 and "config 4" in r.stderr


def test_spawn_refuses_more_gpus_than_visible():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK",
                                                            "HZ_BENCH_REHEARSAL")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "64"], capture_output=True,
                       text=True, timeout=300, cwd=ROOT, env=env)
    assert r.returncode != 0 and "GPU(s) visible" in r.stderr
