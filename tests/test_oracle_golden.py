"""Pins the CPU oracle (oracle/hz_oracle.c) against fixtures captured from the
reference itself (tests/golden/make_golden.py).  CPU only."""
import os

import numpy as np
import pytest

import oracle
from conftest import GOLDEN


def load(name):
    return np.load(os.path.join(GOLDEN, name))


def test_mt_stream_matches_cpython():
    f = load("mt_streams.npz")
    for i, seed in enumerate(f["seeds"]):
        m = oracle.mt_seed(int(seed))
        got = np.array([oracle.mt_next32(m) for _ in range(1000)], np.uint32)
        assert (got == f["words"][i]).all(), f"seed {seed}"


def test_sample_matches_cpython():
    f = load("mt_streams.npz")
    for i, seed in enumerate(f["seeds"]):
        m = oracle.mt_seed(int(seed))
        for j, n in enumerate(f["sample_n"]):
            assert list(oracle.sample(m, int(n), 3)) == list(f["sample"][i, j])
        assert oracle.mt_next32(m) == f["next_word"][i]
        m = oracle.mt_seed(int(seed))
        for n in range(1, 22):
            k = min(3, n)
            assert list(oracle.sample(m, n, k)) == list(f["small_sample"][i, n - 1, :k])


def test_env_traces_bit_exact():
    f = load("env_traces.npz")
    states, masks, acts, off = f["states"], f["masks"], f["actions"], f["offsets"]
    for g, seed in enumerate(f["seeds"]):
        m = oracle.mt_seed(int(seed))
        st = oracle.reset(m)
        for p in range(off[g], off[g + 1]):
            assert (st == states[p]).all(), (seed, p - off[g])
            mask = oracle.legal(st)
            assert (np.packbits(mask, bitorder="little") == masks[p]).all()
            k = oracle.rule(int(seed), p - off[g])
            L = int(mask.sum())
            a = np.flatnonzero(mask)[((k >> 32) * L) >> 32]
            assert a == acts[p]
            r, st = oracle.step(st, int(a), m)
            assert r == 0
        assert (st == f["finals"][g]).all()
        assert oracle.is_game_over(st)
        assert oracle.mt_next32(m) == f["next_word"][g]


def test_env_finals_batch_driver():
    f = load("env_finals.npz")
    seeds = f["seeds"]
    assert (np.diff(seeds) == 1).all()
    total, finals, plies, nxt = oracle.play_rule_games(len(seeds), int(seeds[0]), nthreads=4)
    assert (finals == f["finals"]).all()
    assert (plies == f["plies"]).all()
    assert (nxt == f["next_word"]).all()
    assert total == int(f["plies"].sum())


def test_encoder_matches_reference():
    f = load("encoder.npz")
    for st, b, g in zip(f["states"], f["boards"], f["globs"]):
        ob, og = oracle.encode(st)
        assert (ob.view(np.uint32) == b.view(np.uint32)).all()
        assert (og.view(np.uint32) == g.view(np.uint32)).all()


def test_scoring_known_answers():
    f = load("scoring.npz")
    for b, s in zip(f["boards"], f["scores"]):
        assert list(oracle.score_board(b)) == list(s)
    assert list(f["scores"][0]) == [4, 4, 5, 5, 5]


def test_illegal_moves_report_status():
    m = oracle.mt_seed(0)
    st = oracle.reset(m)
    assert oracle.step(st, 7, m)[0] == 1          # placement index during choose_pile
    assert oracle.step(st, 5 + 0, m)[0] == 1
    r, st1 = oracle.step(st, 0, m)
    assert r == 0
    assert oracle.step(st1, 0, m)[0] == 2         # pile index during placement
    hand = set(int(t) for t in st1[62:62 + st1[65]])
    missing = [t for t in range(6) if t not in hand][0]
    assert oracle.step(st1, 5 + missing * 23, m)[0] == 3
    done = st1.copy()
    done[73] = 4
    assert oracle.step(done, 0, m)[0] == 5


@pytest.mark.parametrize("k", range(80))
def test_mcts_matches_reference(k):
    f = load("mcts.npz")
    m = oracle.mt_seed(int(f["mt_seed"][k]))
    a, visits, nn, ne = oracle.mcts_search(
        f["state"][k], m, int(f["sims"][k]), float(f["cpuct"][k]), eps=float(f["eps"][k]),
        testing=bool(f["testing"][k]), tau0=int(f["tau0"][k]), ply=int(f["ply"][k]),
        u=float(f["u"][k]), noise=f["noise"][k])
    assert (visits == f["visits"][k]).all()
    assert a == f["action"][k]
    assert (nn, ne) == (f["n_nodes"][k], f["n_edges"][k])
    assert oracle.mt_next32(m) == f["next_word"][k]


def test_greedy_games_match_reference():
    """evaluation.choose_move_greedy games (greedy.npz): every state, every
    chosen action, the final state and the next CPython word — the greedy
    agent's simulated apply_move calls consume `random` like real moves."""
    f = np.load(os.path.join(GOLDEN, "greedy.npz"))
    off = f["offsets"]
    for g in range(len(f["seeds"])):
        m = oracle.mt_seed(int(f["seeds"][g]))
        s = oracle.reset(m)
        for p in range(off[g], off[g + 1]):
            assert (s == f["states"][p]).all(), (g, p - off[g])
            a = oracle.greedy_move(s, m)
            assert a == f["actions"][p], (g, p - off[g])
            r, s = oracle.step(s, a, m)
            assert r == 0
        assert (s == f["finals"][g]).all() and oracle.is_game_over(s)
        assert oracle.mt_next32(m) == f["next_word"][g]


def test_play_rule_auto_matches_stepwise_loop():
    """or_play_rule_auto (the steady-state auto-reset oracle) equals the
    step-by-step loop over the oracle's primitives (reset, legal, rule, step),
    and its first game equals or_play_rule_games_ep's."""
    n, base, plies = 12, 4321, 170
    total, finals, games, ep = oracle.play_rule_auto(n, base, plies, ep0=2)
    assert total == n * plies
    _, first, first_plies, _ = oracle.play_rule_games(n, base, episode=2)
    for b in range(n):
        left, e, done = plies, 2, 0
        while True:
            seed = base + b + (e << 32)
            m = oracle.mt_seed(seed)
            s = oracle.reset(m)
            ply = 0
            while left > 0 and not oracle.is_game_over(s):
                mask = oracle.legal(s)
                L = int(mask.sum())
                a = np.flatnonzero(mask)[((oracle.rule(seed, ply) >> 32) * L) >> 32]
                s = oracle.step(s, int(a), m)[1]
                ply += 1
                left -= 1
            done += int(oracle.is_game_over(s))
            if e == 2 and oracle.is_game_over(s):
                assert ply == first_plies[b] and (s == first[b]).all()
            if left <= 0:
                break
            e += 1
        assert (finals[b] == s).all() and games[b] == done and ep[b] == e, b


def test_replay_actions_matches_reference_traces():
    """or_replay_actions (the api_caller leg's check: a caller's own moves
    replayed from the same seeds) reproduces the reference's recorded games
    from their action lists, with no-ops and rejected moves mixed in (a
    rejected move leaves the state as it was, like the reference's
    clone-then-commit)."""
    f = load("env_traces.npz")
    acts, off, seeds = f["actions"], f["offsets"], f["seeds"]
    n = len(seeds)
    lens = off[1:] - off[:-1]
    T = int(lens.max())
    clean = np.full((T, n), -1, np.int16)
    for g in range(n):
        clean[:lens[g], g] = acts[off[g]:off[g + 1]]
    total, finals, rej = oracle.replay_actions(seeds.astype(np.uint64), clean)
    assert total == int(lens.sum()) and (rej == 0).all()
    assert (finals == f["finals"]).all()
    # interleave no-op plies and an illegal action (142 never fits the
    # opening's pile phase, and a pile index past the piles never fits later)
    noisy = np.full((3 * T, n), -1, np.int16)
    noisy[1::3] = clean
    noisy[0, :] = 142
    total2, finals2, rej2 = oracle.replay_actions(seeds.astype(np.uint64), noisy)
    assert total2 == total and (rej2 == 1).all() and (finals2 == finals).all()
