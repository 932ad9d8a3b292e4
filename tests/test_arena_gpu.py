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
    capturable = True  # the stub is PyTorch ops only: the arena's searches replay HIP graphs

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


@pytest.mark.parametrize("testing", [True, False])
def test_graph_replayed_search_matches_eager(testing):
    """search(graph=True): simulation 1 eager (it expands the roots, with the
    Dirichlet noise when not testing), simulations 2.. one captured HIP graph
    replayed.  With the real network on both sides of a routed arena batch
    (BatchedPredictor x 2, the arena's evaluator), the visit counts, tree
    sizes and evaluated-row count equal the eager search's."""
    from hzamd.arena import _Routed
    from hzamd.env import BatchedEnv
    from hzamd.mcts import BatchedMCTS, BatchedPredictor
    from hzamd.net import HarmoniesNet
    torch.manual_seed(0)
    pa = BatchedPredictor(HarmoniesNet().eval().to(DEV))
    pb = BatchedPredictor(HarmoniesNet().eval().to(DEV))
    n = 40
    noise = torch.distributions.Dirichlet(torch.full((69,), 0.3)).sample((n,)).double()
    plies = torch.arange(n, device=DEV) % 30
    out = []
    for graph in (False, True):
        env = BatchedEnv(n, seed_base=55, device=DEV)
        env.reset()
        for p in range(30):
            mask, count = env.legal_mask()
            act = env.rule_actions(mask, count)
            env.step(torch.where(plies > p, act, torch.full_like(act, -1)))
        ev = _Routed(pa, pb, (torch.arange(n, device=DEV) % 3) == 0)
        mcts = BatchedMCTS(env, 24)
        v = mcts.search(ev, 2.0, active=~env.done(), noise=None if testing else noise, eps=0.25,
                        testing=testing, graph=graph).clone()
        out.append((v.cpu(), mcts.stats().clone().cpu(), int(mcts.eval_rows.item())))
        _, mt, idx = env.export_state(with_mt=True)
        out[-1] += (mt.cpu(), idx.cpu())
        mcts.close()
        env.close()
    (v0, c0, r0, m0, i0), (v1, c1, r1, m1, i1) = out
    assert int(v0.sum()) > 0
    assert torch.equal(v0, v1) and torch.equal(c0, c1) and r0 == r1
    assert torch.equal(m0, m1) and torch.equal(i0, i1)
