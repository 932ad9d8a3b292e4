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


def test_root_noise_keyed_by_global_board():
    """hz_root_noise: Dirichlet rows over the live children (sum 1, zeros past
    the legal count), u in [0, 1), and every board's draws depend only on
    (seed, global board id, move): the same in a 64-board batch and in a
    32-board batch whose board_base is 32 further on."""
    from hzamd.selfplay import NoiseSource
    g = torch.Generator().manual_seed(3)
    cnt = torch.randint(0, 70, (64,), generator=g, dtype=torch.int32).to(DEV)
    cnt[0], cnt[1] = 0, 69
    a = NoiseSource(1000, DEV)
    noise, u = a.draw(5, cnt, 0.4)
    live = torch.arange(69, device=DEV).unsqueeze(0) < cnt.unsqueeze(1).long()
    assert (noise[~live] == 0).all() and (noise >= 0).all()
    s = noise.sum(1)
    assert torch.allclose(s[cnt > 0], torch.ones_like(s[cnt > 0]), atol=1e-12)
    assert ((u >= 0) & (u < 1)).all()
    b = NoiseSource(1032, DEV)
    n2, u2 = b.draw(5, cnt[32:].contiguous(), 0.4)
    assert torch.equal(n2, noise[32:]) and torch.equal(u2, u[32:])
    n3, _ = a.draw(6, cnt, 0.4)
    assert not torch.equal(n3, noise)


def test_root_noise_is_dirichlet():
    """Moments of Dirichlet(0.4 * 1_L) at L = 10 over 8,192 draws: mean 1/L,
    variance a(a0 - a) / (a0^2 (a0 + 1)) = 0.018, within sampling error."""
    from hzamd.selfplay import NoiseSource
    n, L = 8192, 10
    cnt = torch.full((n,), L, dtype=torch.int32, device=DEV)
    noise, u = NoiseSource(0, DEV).draw(0, cnt, 0.4)
    x = noise[:, :L].double()
    assert abs(x.mean().item() - 0.1) < 0.003
    var = x.var(0).mean().item()
    assert abs(var - 0.018) < 0.0015, var
    assert abs(u.mean().item() - 0.5) < 0.02


@pytest.mark.parametrize("net", [False, True])
def test_selfplay_split_invariant(net):
    """Per-board self-play records do not depend on how boards are split over
    GPUs: 2 x 24 boards (board bases 700, 724) give
    the same states, visit counts, validity and final states, board by
    board, as 1 x 48 (base 700): the root noise is keyed by global board id
    and every evaluator row is computed independently of its batch."""
    from hzamd.mcts import BatchedPredictor, stub_evaluator
    from hzamd.net import TINY, HarmoniesNet
    from hzamd.selfplay import SelfPlay
    cfg = {"num_simulations": 6, "cpuct": 2.0, "testing": False, "turns_until_tau0": 15}
    if net:
        torch.manual_seed(0)
        ev = BatchedPredictor(HarmoniesNet().to(DEV).eval())
    else:
        ev = stub_evaluator
    recs = [SelfPlay(n, ev, cfg, seed_base=base, device=DEV).play() for n, base in ((48, 700), (24, 700), (24, 724))]
    whole, parts = recs[0], recs[1:]
    for k, part in enumerate(parts):
        sl = slice(24 * k, 24 * k + 24)
        T = part["plies"]
        assert torch.equal(part["valid"], whole["valid"][:T, sl]) and not whole["valid"][T:, sl].any()
        assert torch.equal(part["states"], whole["states"][:T, :, sl])
        assert torch.equal(part["visits"], whole["visits"][:T, sl])
        assert torch.equal(part["final"], whole["final"][:, sl])


@pytest.mark.parametrize("testing", [False, True])
def test_selfplay_steady_matches_oracle_replay(testing):
    """play_steady (continuous self-play: a finished board starts its next
    game, seeded seed_base + b + (k << 32), before the next move) replayed
    board by board by the oracle across game boundaries: every recorded
    state, game index, visit vector, move, game end and outcome; then
    compact_steady's examples (records of ended games only) carry the z
    of the reference's self_play_worker (trainer.py:517-527)."""
    from hzamd.mcts import stub_evaluator
    from hzamd.selfplay import SelfPlay
    n, base, sims, cpuct, tau0, M = 16, 4400, 6, 2.0, 15, 150
    cfg = {"num_simulations": sims, "cpuct": cpuct, "testing": testing, "turns_until_tau0": tau0}
    sp = SelfPlay(n, stub_evaluator, cfg, seed_base=base, device=DEV)
    sp.keep_noise = True
    rec = sp.play_steady(M)
    states, visits = rec["states"].cpu().numpy(), rec["visits"].cpu().numpy()
    game, ended = rec["game"].cpu().numpy(), rec["ended"].cpu().numpy()
    outc = rec["outcome"].cpu().numpy()
    log = [tuple(t.cpu().numpy() for t in x) for x in sp.noise_log]
    assert len(log) == M
    z_want, lengths, n_games = {}, [], 0
    for b in range(n):
        k, ply = 0, 0
        m = oracle.mt_seed(base + b)
        s = oracle.reset(m)
        players = []
        for mv in range(M):
            assert game[mv, b] == k and (unpack_ref(states[mv, :, b]) == s).all(), (b, mv)
            noise, u, act = log[mv]
            a, ov, _, _ = oracle.mcts_search(s, m, sims, cpuct, testing=testing, tau0=tau0, ply=ply,
                                             u=float(u[b]), noise=noise[b])
            assert (visits[mv, b] == ov).all() and a == act[b], (b, mv)
            players.append((mv, int(s[72])))
            r, s = oracle.step(s, a, m)
            assert r == 0
            ply += 1
            if oracle.is_game_over(s):
                w = int(s[75])
                o = 1.0 if w == 0 else -1.0 if w == 1 else 0.0
                assert ended[mv, b] and outc[mv, b] == o, (b, mv)
                for mm, p in players:
                    z_want[(mm, b)] = o if p == 0 else -o
                lengths.append(ply)
                n_games += 1
                players, k, ply = [], k + 1, 0
                m = oracle.mt_seed(base + b + (k << 32))
                s = oracle.reset(m)
            else:
                assert not ended[mv, b], (b, mv)
    assert n_games >= 2 * n  # every board finished at least two games
    comp = sp.compact_steady(rec)
    order = sorted(z_want)  # (move, board): compact's order
    assert comp["z"].shape[0] == len(order)
    assert np.array_equal(comp["z"].cpu().numpy(), np.array([z_want[k] for k in order], np.float32))
    assert np.array_equal(comp["board"].cpu().numpy(), np.array([b for _, b in order]))
    assert sorted(comp["lengths"].cpu().tolist()) == sorted(lengths)
