"""End-to-end parity of batched self-play (hzamd.selfplay) with the C
oracle replaying the same games: every recorded state, every root visit
vector, every move and the final state, with the search's chance draws and
the real moves' draws interleaved on each board's CPython stream exactly as
in self_play_worker (trainer.py:468-509)."""
import numpy as np
import pytest
import torch

import oracle
from hzamd.state import unpack_ref

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def replay(rec, sp, n, base, sims, cpuct, testing, tau0):
    """Replays every board's game with the oracle; returns the expected z of
    every record in SelfPlay.compact's order (trainer.py:517-527: the final
    outcome from the recorded player's perspective, 0 for a draw)."""
    states = rec["states"].cpu().numpy()
    visits = rec["visits"].cpu().numpy()
    valid = rec["valid"].cpu().numpy()
    log = sp.noise_log
    final = rec["final"].cpu().numpy()
    z = np.zeros(valid.shape, np.float32)
    for b in range(n):
        m = oracle.mt_seed(base + b)
        s = oracle.reset(m)
        ply = 0
        while not oracle.is_game_over(s):
            assert valid[ply, b]
            assert (unpack_ref(states[ply, :, b]) == s).all(), (b, ply)
            noise, u, act = (t.cpu().numpy() for t in log[ply])
            a, ov, _, _ = oracle.mcts_search(s, m, sims, cpuct, testing=testing, tau0=tau0, ply=ply,
                                             u=float(u[b]), noise=noise[b])
            assert (visits[ply, b] == ov).all(), (b, ply)
            assert a == act[b], (b, ply)
            r, s = oracle.step(s, a, m)
            assert r == 0
            ply += 1
        assert (unpack_ref(final[:, b]) == s).all(), b
        assert not valid[ply:, b].any()
        w = int(s[75])                                    # winner: 0 / 1, negative = draw
        outcome = 1.0 if w == 0 else -1.0 if w == 1 else 0.0
        for p in range(ply):
            player = int(unpack_ref(states[p, :, b])[72])
            z[p, b] = outcome if player == 0 else -outcome
    return z[valid]


@pytest.mark.parametrize("testing", [True, False])
def test_selfplay_matches_oracle_replay(testing):
    from hzamd.mcts import stub_evaluator
    from hzamd.selfplay import SelfPlay
    n, base, sims, cpuct = 24, 900, 6, 2.0
    cfg = {"num_simulations": sims, "cpuct": cpuct, "testing": testing, "turns_until_tau0": 15}
    sp = SelfPlay(n, stub_evaluator, cfg, seed_base=base, device=DEV)
    sp.keep_noise = True
    rec = sp.play()
    z_want = replay(rec, sp, n, base, sims, cpuct, testing, 15)
    comp = sp.compact(rec)
    assert comp["states"].shape[0] == int(rec["valid"].sum())
    assert np.array_equal(comp["z"].cpu().numpy(), z_want)
    assert (z_want != 0).any()
    assert torch.allclose(comp["pi"].sum(1), torch.ones(comp["pi"].shape[0], device=comp["pi"].device))
    ex = sp.examples(comp)
    assert ex[0][0].shape == (38, 5, 7) and ex[0][1].shape == (42,) and ex[0][2].shape == (143,)
    assert ex[0][3].shape == (1,)


def test_selfplay_with_network_runs():
    """Default-architecture network (model.py:277-394 restated), random init:
    self-play completes and yields well-formed examples."""
    from hzamd.mcts import BatchedPredictor
    from hzamd.net import TINY, HarmoniesNet
    from hzamd.selfplay import SelfPlay
    torch.manual_seed(0)
    net = HarmoniesNet(TINY).to(DEV).eval()
    sp = SelfPlay(64, BatchedPredictor(net), {"num_simulations": 4, "cpuct": 1.0}, seed_base=3, device=DEV)
    rec = sp.play()
    comp = sp.compact(rec)
    z = comp["z"].cpu().numpy()
    assert set(np.unique(z)).issubset({-1.0, 0.0, 1.0})
    out = sp.outcomes(rec["final"]).cpu().numpy()
    assert (np.abs(out) <= 1).all()
