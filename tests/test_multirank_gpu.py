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


def _loop(tmp_path, tag, nproc, port, backend="gloo"):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(ROOT, "tests", "dist_loop_rehearsal.py"), str(tmp_path / tag), str(tmp_path / f"run_{tag}")]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT,
                       env=dict(os.environ, HZ_DIST_BACKEND=backend))
    assert r.returncode == 0, r.stderr[-3000:]
    return [torch.load(tmp_path / f"{tag}.rank{k}.pt", weights_only=True) for k in range(nproc)]


def test_training_loop_rccl_one_rank_equals_gloo(tmp_path):
    """The loop's collectives on RCCL (one rank: records all-gather on device
    tensors, weight broadcast, arena all-reduce) end with the same weights,
    best weights, replay buffer and decisions as the same loop over gloo.
    The rehearsal trains in a fixed summation order (HZ_DETERMINISTIC: no
    MIOpen, deterministic algorithms), so the weights after the broadcasts
    are compared bit for bit."""
    (a,) = _loop(tmp_path, "rccl", 1, 29527, "nccl")
    (b,) = _loop(tmp_path, "gloo", 1, 29529, "gloo")
    assert a["backend"] == "nccl" and b["backend"] == "gloo"
    assert torch.equal(a["buffer"], b["buffer"]) and a["examples"] == b["examples"]
    for k in ("model", "best"):
        assert torch.isfinite(a[k]).all(), k
        assert torch.equal(a[k], b[k]), (k, float((a[k] - b[k]).abs().max()))
    assert a["evals"] == b["evals"] and a["evals"][1] is not None


def test_training_loop_two_ranks(tmp_path):
    a, b = _loop(tmp_path, "out", 2, 29523)
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
