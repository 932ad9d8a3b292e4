"""The torch stub evaluator (hzamd.mcts.stub_evaluator) equals the golden
stub (tests/golden/make_golden.py) and the oracle's C restatement. CPU only."""
import os

import numpy as np
import torch

import oracle
from conftest import GOLDEN


def test_stub_evaluator_matches_oracle_stub():
    from hzamd.mcts import stub_evaluator
    f = np.load(os.path.join(GOLDEN, "env_traces.npz"))
    states = f["states"][::11]
    boards, globs = zip(*[oracle.encode(s) for s in states])
    pol, val = stub_evaluator(torch.from_numpy(np.stack(boards)), torch.from_numpy(np.stack(globs)))
    for i, s in enumerate(states):
        op, ov = oracle.stub_eval(s)
        assert (pol[i].numpy() == op).all()
        assert float(val[i]) == ov


def test_choose_actions_rules():
    from hzamd.mcts import choose_actions, pi_from_visits
    v = torch.tensor([[0, 3, 5, 5, 0], [2, 0, 2, 1, 0], [0, 0, 0, 0, 0]], dtype=torch.int32)
    g = choose_actions(v, torch.zeros(3, dtype=torch.bool), torch.zeros(3))
    assert g.tolist() == [2, 0, -1]          # first maximum
    e = choose_actions(v, torch.ones(3, dtype=torch.bool), torch.tensor([0.0, 0.5, 0.3], dtype=torch.float64))
    assert e.tolist() == [1, 2, -1]          # 0*13 < 3 -> 1; 0.5*5 = 2.5 < cum 4 -> 2
    p = pi_from_visits(v)
    assert torch.allclose(p[0], torch.tensor([0, 3, 5, 5, 0]) / 13.0)
