"""Batched greedy agent (hz_greedy_actions, evaluation.py:137-196) against
the reference's greedy-vs-greedy games (tests/golden/greedy.npz) and the C
oracle at 1024 boards: actions, every state and the chance streams bit-exact."""
import os

import numpy as np
import pytest
import torch

import oracle
from conftest import GOLDEN
from hzamd.state import unpack_ref

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def states_of(env):
    st = env.export_state().cpu().numpy()
    return np.stack([unpack_ref(st[:, b]) for b in range(env.n)])


def test_greedy_games_match_reference_fixtures():
    from hzamd.env import BatchedEnv
    f = np.load(os.path.join(GOLDEN, "greedy.npz"))
    off = f["offsets"]
    G = len(f["seeds"])
    env = BatchedEnv(G, device=DEV)
    env.reset(seeds=torch.tensor(f["seeds"].astype(np.int64), device=DEV))
    ply = 0
    while True:
        st = states_of(env)
        act = env.greedy_actions().cpu().numpy()
        live = [g for g in range(G) if off[g] + ply < off[g + 1]]
        if not live:
            assert (act == -1).all()
            break
        for g in range(G):
            if off[g] + ply < off[g + 1]:
                assert (st[g] == f["states"][off[g] + ply]).all(), (g, ply)
                assert act[g] == f["actions"][off[g] + ply], (g, ply)
            else:
                assert act[g] == -1 and (st[g] == f["finals"][g]).all(), (g, ply)
        status = env.step(torch.from_numpy(act).to(DEV))
        assert (status.cpu().numpy()[live] == 0).all()
        ply += 1
    assert (states_of(env) == f["finals"]).all()
    _, mt, idx = env.export_state(with_mt=True)
    mt, idx = mt.cpu().numpy().view(np.uint32), idx.cpu().numpy()
    for g in range(G):
        assert oracle.mt_next32(oracle.mt_from_words(mt[g], idx[g])) == f["next_word"][g]


def test_greedy_1024_boards_vs_oracle():
    from hzamd.env import BatchedEnv
    n, base = 1024, 7000
    env = BatchedEnv(n, seed_base=base, device=DEV)
    env.reset()
    for _ in range(200):
        act = env.greedy_actions()
        if bool((act < 0).all()):
            break
        env.step(act)
    got = states_of(env)
    _, mt, idx = env.export_state(with_mt=True)
    mt, idx = mt.cpu().numpy().view(np.uint32), idx.cpu().numpy()
    for b in range(n):
        m = oracle.mt_seed(base + b)
        s = oracle.reset(m)
        while not oracle.is_game_over(s):
            s = oracle.step(s, oracle.greedy_move(s, m), m)[1]
        assert (got[b] == s).all(), b
        if b % 64 == 0:
            assert oracle.mt_next32(oracle.mt_from_words(mt[b], idx[b])) == oracle.mt_next32(m), b
