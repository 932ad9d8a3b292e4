"""Arena bookkeeping that needs no GPU: the reference's win-rate rule
(trainer.py:333-338: wins / decisive games, 0.5 without decisive games) and
the evaluation-agent guard."""
import pytest
import torch

from hzamd.arena import MctsAgent, summarize


def test_summarize_win_rate():
    s = summarize(torch.tensor([1, -1, 0, 1, 1]))
    assert (s["wins"], s["losses"], s["draws"]) == (3, 1, 1) and s["win_rate"] == 0.75
    assert summarize(torch.tensor([0, 0]))["win_rate"] == 0.5


def test_eval_agent_is_deterministic_search():
    with pytest.raises(ValueError):
        MctsAgent(lambda b, g: None, {"testing": False})
    with pytest.raises(ValueError):
        MctsAgent(lambda b, g: None, {"dirichlet_epsilon": 0.25})
