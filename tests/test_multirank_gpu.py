"""The multi-rank training loop (BASELINE config 5) rehearsed at world 2
over gloo with both ranks on this box's GPU (tests/dist_loop_rehearsal.py):
after self-play -> all-gather -> rank-0 training -> weight broadcast ->
checkpoint -> sharded arena, both ranks hold identical weights, identical
replay buffers and took the same promotion decision (trainer.py:62-375)."""
import os
import subprocess
import sys

import pytest
import torch

from conftest import ROOT

pytestmark = pytest.mark.gpu


def test_training_loop_two_ranks(tmp_path):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29523",
           os.path.join(ROOT, "tests", "dist_loop_rehearsal.py"), str(tmp_path / "out"), str(tmp_path / "run")]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    a, b = (torch.load(tmp_path / f"out.rank{k}.pt", weights_only=True) for k in (0, 1))
    assert a["world"] == b["world"] == 2
    assert torch.equal(a["model"], b["model"])
    assert torch.equal(a["best"], b["best"])
    assert torch.equal(a["buffer"], b["buffer"]) and a["buffer"].shape[0] == min(1000, sum(a["examples"]))
    assert a["evals"] == b["evals"]
    e = a["evals"][1]
    assert e is not None and e["wins"] + e["losses"] + e["draws"] == 5
    # threshold 0: the candidate is promoted unless it lost every decisive game
    if e["passed"]:
        assert torch.equal(a["best"], a["model"])
