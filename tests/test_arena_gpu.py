"""Batched evaluation games (hzamd.arena): greedy vs greedy, MCTS vs greedy
(evaluation.run_tournament) and MCTS vs MCTS with routed leaf batches
(Trainer.evaluate_model), every game replayed by the C oracle — final states
bit-exact, outcomes from agent A's perspective."""
import numpy as np
import pytest
import torch

import oracle
from hzamd.arena import GreedyAgent, MctsAgent, play_games, summarize
from hzamd.mcts import stub_evaluator
from hzamd.state import unpack_ref

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
SIMS = 8


def oracle_game(seed, a_is_p0, agent_a, agent_b):
    m = oracle.mt_seed(seed)
    s = oracle.reset(m)
    ply = 0
    while not oracle.is_game_over(s):
        a_turn = (int(s[72]) == 0) == a_is_p0
        kind = agent_a if a_turn else agent_b
        if kind == "greedy":
            a = oracle.greedy_move(s, m)
        else:
            a = oracle.mcts_search(s, m, SIMS, 2.0, eps=0.0, testing=True, tau0=0, ply=ply,
                                   negate_value=kind == "mcts_neg")[0]
        s = oracle.step(s, a, m)[1]
        ply += 1
    return s


def check(agent_a, agent_b, kinds, n, base):
    outcome, final, _ = play_games(agent_a, agent_b, n, seed_base=base, device=DEV)
    fin = final.cpu().numpy()
    for g in range(n):
        s = oracle_game(base + g, g % 2 == 0, *kinds)
        assert (unpack_ref(fin[:, g]) == s).all(), g
        w = int(s[75])
        o = 0 if w in (-1, -2) else (1 if w == 0 else -1)
        assert int(outcome[g]) == (o if g % 2 == 0 else -o), g
    return outcome


def test_greedy_vs_greedy():
    check(GreedyAgent(), GreedyAgent(), ("greedy", "greedy"), 64, 300)


def test_mcts_vs_greedy_tournament():
    a = MctsAgent(stub_evaluator, {"num_simulations": SIMS})
    out = check(a, GreedyAgent(), ("mcts", "greedy"), 16, 400)
    s = summarize(out)
    assert s["wins"] + s["losses"] + s["draws"] == 16


def neg_stub_evaluator(board, glob):
    p, v = stub_evaluator(board, glob)
    return p, -v


def test_mcts_vs_mcts_routed_batch():
    a = MctsAgent(stub_evaluator, {"num_simulations": SIMS})
    b = MctsAgent(stub_evaluator, {"num_simulations": SIMS})
    check(a, b, ("mcts", "mcts"), 16, 500)


class _DeviceRows:
    """A device-row evaluator (as BatchedPredictor): called on the whole
    gathered buffers with the live count left on the device."""

    device_rows = True

    def __init__(self, fn):
        self.fn = fn

    def __call__(self, board, glob, rows=None, count=None):
        return self.fn(board, glob)


def test_mcts_vs_mcts_routed_device_rows_two_evaluators():
    """The no-round-trip routing (both evaluators on the whole gathered
    batch, rows picked by their board's agent) plays the same games as the
    oracle with each agent's own evaluator."""
    a = MctsAgent(_DeviceRows(stub_evaluator), {"num_simulations": SIMS})
    b = MctsAgent(_DeviceRows(neg_stub_evaluator), {"num_simulations": SIMS})
    check(a, b, ("mcts", "mcts_neg"), 24, 700)


def test_mcts_vs_mcts_routed_batch_two_evaluators():
    """The shared search routes each gathered leaf row to its board's agent
    by board id: two different evaluators (the stub and its negated value),
    games ending at different plies (the gathered batch shrinks and shifts),
    every game replayed by the oracle with each agent's own evaluator."""
    a = MctsAgent(stub_evaluator, {"num_simulations": SIMS})
    b = MctsAgent(neg_stub_evaluator, {"num_simulations": SIMS})
    out = check(a, b, ("mcts", "mcts_neg"), 24, 600)
    s = summarize(out)
    assert s["wins"] + s["losses"] + s["draws"] == 24
