"""GPU parity of the HIP env kernels (libhz.so via hzamd.BatchedEnv) against
the reference golden fixtures and the C oracle.  Bit-exact for every state,
mask, action, score and encoder output."""
import os

import numpy as np
import pytest
import torch

import oracle
from conftest import GOLDEN
from hzamd.state import pack_ref, unpack_ref, words_to_array

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def load(name):
    return np.load(os.path.join(GOLDEN, name))


@pytest.fixture(scope="module")
def Env():
    from hzamd.env import BatchedEnv
    return BatchedEnv


def states_of(env):
    st = env.export_state().cpu().numpy()
    return np.stack([unpack_ref(st[:, b]) for b in range(env.n)])


def import_refstates(env, refs):
    words = words_to_array([pack_ref(v) for v in refs])  # [n, 6]
    env.import_state(torch.from_numpy(np.ascontiguousarray(words.T)))


def mask_bits(mask_words):
    """int64 [n,3] -> uint8 [n,143]"""
    m = mask_words.view(np.uint64) if mask_words.dtype == np.int64 else mask_words
    out = np.zeros((m.shape[0], 143), np.uint8)
    for a in range(143):
        out[:, a] = (m[:, a // 64] >> np.uint64(a % 64)) & np.uint64(1)
    return out


def test_reset_matches_reference(Env):
    f = load("env_traces.npz")
    env = Env(64, seed_base=0, device=DEV)
    env.reset()
    got = states_of(env)
    first = f["states"][f["offsets"][:-1]]
    assert (got == first).all()


def test_stepwise_api_matches_traces(Env):
    """legal_mask -> rule_actions -> step, ply by ply, against the traces."""
    f = load("env_traces.npz")
    off = f["offsets"]
    n = len(f["seeds"])
    env = Env(n, seed_base=0, device=DEV)
    env.reset()
    ply = 0
    max_len = int(np.diff(off).max())
    while ply < max_len:
        live = np.array([off[g] + ply < off[g + 1] for g in range(n)])
        mask, count = env.legal_mask()
        acts = env.rule_actions(mask, count)
        st = states_of(env)
        mb = mask_bits(mask.cpu().numpy())
        a = acts.cpu().numpy()
        for g in range(n):
            if live[g]:
                p = off[g] + ply
                assert (st[g] == f["states"][p]).all(), (g, ply)
                assert (np.packbits(mb[g], bitorder="little") == f["masks"][p]).all(), (g, ply)
                assert a[g] == f["actions"][p], (g, ply)
            else:
                assert a[g] == -1 and mb[g].sum() == 0
        status = env.step(acts).cpu().numpy()
        assert (status[live] == 0).all()
        assert (status[~live] == 7).all()
        ply += 1
    st = states_of(env)
    assert (st == f["finals"]).all()
    assert env.done().all()


def test_rollout_records_traces(Env):
    f = load("env_traces.npz")
    off = f["offsets"]
    n = len(f["seeds"])
    env = Env(n, seed_base=0, device=DEV)
    env.reset()
    games, steps, (ts, tm, ta) = env.rollout(max_plies=80, record=True)
    ts, tm, ta = ts.cpu().numpy(), tm.cpu().numpy(), ta.cpu().numpy()
    assert (steps.cpu().numpy() == f["plies"]).all()
    assert (games.cpu().numpy() == 1).all()
    for g in range(n):
        L = off[g + 1] - off[g]
        for ply in range(L):
            p = off[g] + ply
            assert (unpack_ref(ts[ply, :, g]) == f["states"][p]).all()
            assert (np.packbits(mask_bits(tm[ply, g][None])[0], bitorder="little") == f["masks"][p]).all()
            assert ta[ply, g] == f["actions"][p]
        assert (ta[L:, g] == -1).all()
    assert (states_of(env) == f["finals"]).all()


def test_rollout_finals_and_rng_stream(Env):
    f = load("env_finals.npz")
    n = len(f["seeds"])
    env = Env(n, seed_base=int(f["seeds"][0]), device=DEV)
    env.reset()
    games, steps, _ = env.rollout(max_plies=200)
    assert (steps.cpu().numpy() == f["plies"]).all()
    assert (states_of(env) == f["finals"]).all()
    _, mt, idx = env.export_state(with_mt=True)
    mt = mt.cpu().numpy().view(np.uint32)
    idx = idx.cpu().numpy()
    for b in range(n):
        m = oracle.mt_from_words(mt[b], idx[b])
        assert oracle.mt_next32(m) == f["next_word"][b], b


def test_full_size_4096_vs_oracle(Env):
    """BASELINE config 2 size: 4096 boards to game end, bit-exact vs the C oracle."""
    n, base = 4096, 777
    env = Env(n, seed_base=base, device=DEV)
    env.reset()
    games, steps, _ = env.rollout(max_plies=200)
    total, finals, plies, nxt = oracle.play_rule_games(n, base, nthreads=8)
    assert (states_of(env) == finals).all()
    assert (steps.cpu().numpy() == plies).all()
    assert int(steps.sum()) == total
    score = env.score().cpu().numpy()
    assert (score[:, 0] == finals[:, 76]).all() and (score[:, 1] == finals[:, 77]).all()


def test_fused_play_and_staged_continue(Env):
    """hz_play (reset fused into the rollout, streams seeded in LDS) and a
    rollout continued from mid-game (streams staged HBM -> LDS -> HBM)."""
    n, base = 4096, 4321
    env = Env(n, seed_base=base, device=DEV)
    games, steps, _ = env.rollout(21, reset=True)
    assert (games.cpu().numpy() == 0).all() and (steps.cpu().numpy() == 21).all()
    games2, steps2, _ = env.rollout(200)
    total, finals, plies, nxt = oracle.play_rule_games(n, base, nthreads=8)
    assert (states_of(env) == finals).all()
    assert ((steps.cpu().numpy() + steps2.cpu().numpy()) == plies).all()
    _, mt, idx = env.export_state(with_mt=True)
    mt, idx = mt.cpu().numpy().view(np.uint32), idx.cpu().numpy()
    for b in range(0, n, 97):
        assert oracle.mt_next32(oracle.mt_from_words(mt[b], idx[b])) == nxt[b]


def _check_episode(env, base, ep, steps, nthreads=8):
    total, finals, plies, nxt = oracle.play_rule_games(env.n, base, nthreads=nthreads, episode=ep)
    assert (states_of(env) == finals).all(), ep
    assert (steps.cpu().numpy() == plies).all(), ep
    _, mt, idx = env.export_state(with_mt=True)
    mt, idx = mt.cpu().numpy().view(np.uint32), idx.cpu().numpy()
    for b in range(0, env.n, 131):
        assert oracle.mt_next32(oracle.mt_from_words(mt[b], idx[b])) == nxt[b], (ep, b)


@pytest.mark.parametrize("ahead,draws", [(True, 24), (True, 3), (True, 16), (True, 19), (False, 0)])
def test_play_seed_ahead_pipeline(Env, ahead, draws):
    """Consecutive hz_play calls (episodes 0-4: the first three fill the
    seed -> draw1 -> draw2 pipeline, the rest replay fully prepared slots),
    an hz_reset + hz_rollout in between (episode 5, re-primes the pipeline;
    the ring slots then hold stale episodes), then episodes 6-10: every game
    bit-exact vs the oracle's episode.  draws < 19 makes every game (19-23
    draws) run past its pile script onto the prepared stream; 19 covers the
    boundary; 16 leaves draw2 nothing to draw."""
    n, base = 4096, 2024
    env = Env(n, seed_base=base, device=DEV)
    env.set_pipeline(1)
    env.set_seed_ahead(ahead, draws)
    for ep in range(5):
        _, steps, _ = env.rollout(200, reset=True)
        _check_episode(env, base, ep, steps)
    env.reset()
    _, steps, _ = env.rollout(200)
    _check_episode(env, base, 5, steps)
    for ep in range(6, 11):
        _, steps, _ = env.rollout(200, reset=True)
        _check_episode(env, base, ep, steps)


@pytest.mark.parametrize("draws", [24, 19, 3, 0])
def test_play_pipeline2(Env, draws):
    """hz_play's second pipeline (k_play2: seeding pass 1 in two stages, pass
    2 in three, four draw stages, four play stages, one stage per call on
    thirteen episodes at once): sixteen consecutive calls (the first twelve
    fill the stages, from the thirteenth every board replays a fully
    prepared episode), an hz_reset + hz_rollout (re-primes: the hand-off
    slots then hold stale episodes), then sixteen more calls; every game, ply count and
    stream bit-exact vs the oracle's episode.  draws < 19 runs games past
    their pile scripts onto the stream slots; 0 prepares no script at all."""
    n, base = 4096, 4242
    env = Env(n, seed_base=base, device=DEV)
    env.set_pipeline(2)
    env.set_seed_ahead(draws > 0, draws)
    for ep in range(16):
        _, steps, _ = env.rollout(200, reset=True)
        _check_episode(env, base, ep, steps)
    env.reset()
    _, steps, _ = env.rollout(200)
    _check_episode(env, base, 16, steps)
    for ep in range(17, 33):
        _, steps, _ = env.rollout(200, reset=True)
        _check_episode(env, base, ep, steps)
    env.check_errors()  # no wait gave up


@pytest.mark.parametrize("pipeline", [2, 1])
def test_play_wait_give_up_is_loud(pipeline):
    """The pipelines' bounded waits (k_play2's twist wave following P2c, the
    chance-ahead seed stage's writers following wave 0) report giving up:
    with the spin bound forced to one round the waits give up, the env's
    error word is set and check_errors() raises NativeError; with the
    default bound (and after the error was taken) nothing is raised."""
    from hzamd._native import NativeError
    from hzamd.env import BatchedEnv
    env = BatchedEnv(512, seed_base=5, device=DEV)
    env.set_pipeline(pipeline)
    for _ in range(3):
        env.rollout(200, reset=True)
    env.check_errors()
    env.set_spin_limit(1)
    with pytest.raises(NativeError, match="gave up waiting"):
        for _ in range(14):
            env.rollout(200, reset=True)
        env.check_errors()
    env.set_spin_limit(0)
    torch.cuda.synchronize()
    env.wait_err.zero_()
    env.reset()
    for _ in range(3):
        env.rollout(200, reset=True)
    env.check_errors()
    env.close()


def test_play_pipeline2_partial_block_and_switch(Env):
    """Pipeline 2 with a partial block (1000 boards), switched to pipeline 1
    and back mid-stream (each pipeline's hand-offs go stale while the other
    runs), and after an auto-reset call that moves counters board by board."""
    n, base = 1000, 99
    env = Env(n, seed_base=base, device=DEV)
    env.set_pipeline(2)
    ep = 0
    for pipe, calls in ((2, 15), (1, 2), (2, 15)):
        env.set_pipeline(pipe)
        for _ in range(calls):
            _, steps, _ = env.rollout(200, reset=True)
            _check_episode(env, base, ep, steps)
            ep += 1
    games, _, _ = env.rollout(64, auto_reset=True, reset=True)  # episode ep, then maybe ep + 1
    resets = games.cpu().numpy() - env.done().cpu().numpy().astype(np.int64)
    nxt_ep = ep + 1 + resets
    _, steps, _ = env.rollout(200, reset=True)
    st = states_of(env)
    steps = steps.cpu().numpy()
    for e in sorted(set(nxt_ep.tolist())):
        _, finals, plies, _ = oracle.play_rule_games(n, base, nthreads=8, episode=int(e))
        sel = nxt_ep == e
        assert (st[sel] == finals[sel]).all(), e
        assert (steps[sel] == plies[sel]).all(), e


def test_play_pipeline_partial_block(Env):
    """hz_play's pipeline with a board count that leaves a partial block
    (1000 = 15 x 64 + 40): ring slots padded to whole blocks, play slots
    unpadded; six consecutive calls (the last three fully prepared), every
    game bit-exact."""
    n, base = 1000, 777
    env = Env(n, seed_base=base, device=DEV)
    env.set_pipeline(1)
    for ep in range(6):
        _, steps, _ = env.rollout(200, reset=True)
        _check_episode(env, base, ep, steps)


@pytest.mark.parametrize("pipeline", [1, 2])
def test_play_after_auto_reset_mispredicts_safely(Env, pipeline):
    """hz_play with auto_reset moves episode counters by a board-dependent
    amount, so the concurrent seed-ahead guesses wrong for some boards: the
    next hz_play must still play every board's true next episode."""
    n, base = 1024, 55
    env = Env(n, seed_base=base, device=DEV)
    env.set_pipeline(pipeline)
    env.rollout(200, reset=True)                                  # episode 0 everywhere
    games, _, _ = env.rollout(64, auto_reset=True, reset=True)    # episode 1, then maybe 2
    resets = games.cpu().numpy() - env.done().cpu().numpy().astype(np.int64)
    nxt_ep = 2 + resets
    assert len(set(nxt_ep.tolist())) > 1
    _, steps, _ = env.rollout(200, reset=True)
    st = states_of(env)
    steps = steps.cpu().numpy()
    for ep in sorted(set(nxt_ep.tolist())):
        _, finals, plies, _ = oracle.play_rule_games(n, base, nthreads=8, episode=int(ep))
        sel = nxt_ep == ep
        assert (st[sel] == finals[sel]).all(), ep
        assert (steps[sel] == plies[sel]).all(), ep


def test_auto_reset_steady_state(Env):
    """auto_reset: board b's k-th game is seeded seed_base + b + (k << 32)."""
    n, base, plies = 256, 31, 150
    env = Env(n, seed_base=base, device=DEV)
    env.reset()
    games, steps, _ = env.rollout(max_plies=plies, auto_reset=True)
    st = states_of(env)
    g = games.cpu().numpy()
    for b in range(0, n, 17):
        left, e, done_games = plies, 0, 0
        s = None
        while left > 0:
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
            done_games += int(oracle.is_game_over(s))
            e += 1
        assert (st[b] == s).all(), b
        assert g[b] == done_games
    assert (steps.cpu().numpy() == plies).all()


def test_scoring_known_answers(Env):
    f = load("scoring.npz")
    boards = f["boards"]
    refs = np.zeros((len(boards), 78), np.int16)
    refs[:, 0:23] = boards
    refs[:, 23:46] = boards[::-1]
    refs[:, 46:61] = -1
    refs[:, 62:65] = -1
    refs[:, 75] = -2
    env = Env(len(boards), device=DEV)
    import_refstates(env, refs)
    total, parts = env.score(parts=True)
    parts = parts.cpu().numpy()
    assert (parts[:, 0, :] == f["scores"]).all()
    assert (parts[:, 1, :] == f["scores"][::-1]).all()
    assert (total.cpu().numpy()[:, 0] == f["scores"].sum(1)).all()
    assert list(parts[0, 0]) == [4, 4, 5, 5, 5]


def test_encoder_bit_exact(Env):
    f = load("encoder.npz")
    refs = f["states"]
    env = Env(len(refs), device=DEV)
    import_refstates(env, refs)
    board, glob = env.encode()
    b = board.cpu().numpy()
    g = glob.cpu().numpy()
    assert (b.view(np.uint32) == f["boards"].view(np.uint32)).all()
    assert (g.view(np.uint32) == f["globs"].view(np.uint32)).all()
    # gathered subset, reversed order
    idx = torch.arange(len(refs) - 1, -1, -3, dtype=torch.int32)
    board2, glob2 = env.encode(idx)
    assert (board2.cpu().numpy() == f["boards"][idx.numpy()]).all()
    assert (glob2.cpu().numpy() == f["globs"][idx.numpy()]).all()


def test_encoder_odd_counts_and_empty_slots(Env):
    """Pairs kernel edge cases: an odd number of states (the last pair holds
    one) and idx < 0 entries (all-zero records, MCTS's inactive boards)."""
    f = load("encoder.npz")
    refs = f["states"]
    env = Env(len(refs), device=DEV)
    import_refstates(env, refs)
    for m in (1, 3, 63, 129):
        idx = torch.arange(m, dtype=torch.int32) * 2 % len(refs)
        idx[1::4] = -1
        board, glob = env.encode(idx)
        b, g = board.cpu().numpy(), glob.cpu().numpy()
        for k in range(m):
            j = int(idx[k])
            if j < 0:
                assert not b[k].any() and not g[k].any(), (m, k)
            else:
                assert (b[k] == f["boards"][j]).all() and (g[k] == f["globs"][j]).all(), (m, k)


@pytest.mark.parametrize("pipeline,calls", [(1, 3), (2, 15)])
def test_play_partial_blocks(Env, pipeline, calls):
    """100 boards (a partial 64-board block in every role of the launch):
    consecutive hz_play calls (pipeline 2: until episodes are fully
    prepared), each bit-exact vs the oracle's episode."""
    n, base = 100, 9
    env = Env(n, seed_base=base, device=DEV)
    env.set_pipeline(pipeline)
    for ep in range(calls):
        _, steps, _ = env.rollout(200, reset=True)
        _check_episode(env, base, ep, steps)


def test_encoder_game_over_states(Env):
    f = load("env_finals.npz")
    refs = f["finals"][:128]
    env = Env(len(refs), device=DEV)
    import_refstates(env, refs)
    board, glob = env.encode()
    for k in range(len(refs)):
        ob, og = oracle.encode(refs[k])
        assert (board[k].cpu().numpy() == ob).all() and (glob[k].cpu().numpy() == og).all()


def test_status_codes_match_reference_errors(Env):
    env = Env(8, seed_base=5, device=DEV)
    env.reset()
    before = env.export_state().clone()
    # choose_pile phase: placement index -> bad pile (1), pile 5 -> bad pile (1),
    # id 143 -> bad action (6), -1 -> no-op (7); the board must not change
    acts = torch.tensor([7, 5, 143, -1, 0, 1, 2, 3], dtype=torch.int16)
    st = env.step(acts).cpu().numpy()
    assert list(st) == [1, 1, 6, 7, 0, 0, 0, 0]
    after = env.export_state()
    assert (after[:, :4] == before[:, :4]).all()
    assert not (after[:, 4:] == before[:, 4:]).all()
    # boards 4..7 are placing: pile index -> bad format (2), missing tile -> 3
    ref = states_of(env)
    acts = [-1, -1, -1, -1]
    for b in range(4, 8):
        hand = set(int(t) for t in ref[b, 62:62 + ref[b, 65]])
        missing = [t for t in range(6) if t not in hand][0]
        acts.append(0 if b < 6 else 5 + missing * 23 + 11)
    st = env.step(torch.tensor(acts, dtype=torch.int16)).cpu().numpy()
    assert list(st[4:]) == [2, 2, 3, 3]
    # illegal stacking (4): second tile on the occupied centre cell when the
    # oracle says so; game_over phase (5)
    for seed in range(40):
        m = oracle.mt_seed(seed)
        s = oracle.reset(m)
        s = oracle.step(s, 0, m)[1]
        hand = [int(t) for t in s[62:65] if t >= 0]
        s = oracle.step(s, 5 + hand[0] * 23 + 11, m)[1]
        blocked = 5 + hand[1] * 23 + 11
        expect, _ = oracle.step(s, blocked, oracle.mt_seed(seed))
        if expect == 4:
            break
    assert expect == 4
    env2 = Env(1, device=DEV)
    import_refstates(env2, [s])
    assert env2.step(torch.tensor([blocked], dtype=torch.int16)).cpu().numpy()[0] == 4
    over = s.copy()
    over[73] = 4
    import_refstates(env2, [over])
    assert env2.step(torch.tensor([0], dtype=torch.int16)).cpu().numpy()[0] == 5


def test_mt_import_export_roundtrip_cpython(Env):
    """A CPython random state imported mid-stream continues exactly like CPython."""
    import random
    r = random.Random(99)
    for _ in range(700):
        r.getrandbits(32)
    ver, words, _ = r.getstate()
    words = np.array(words, np.uint64)
    env = Env(1, device=DEV)
    m = oracle.mt_seed(0)
    st = oracle.reset(m)
    mt = torch.from_numpy(words[:624].astype(np.uint32).view(np.int32).reshape(1, 624).copy())
    idx = torch.tensor([int(words[624])], dtype=torch.int32)
    import_refstates(env, [st])
    env.import_state(env.export_state(), mt, idx)
    _, mt2, idx2 = env.export_state(with_mt=True)
    assert (mt2.cpu().numpy().view(np.uint32)[0] == words[:624]).all()
    assert idx2.item() == int(words[624])
    # and the next draws continue CPython's stream
    acts = torch.tensor([0], dtype=torch.int16)
    m = oracle.mt_from_words(words[:624], int(words[624]))
    s1 = oracle.step(st, 0, m)[1]
    env.step(acts)
    assert (states_of(env)[0] == s1).all()


def test_rule_ply_equals_three_calls():
    """hz_rule_ply (legal mask -> rule pick -> step in one launch) writes, ply
    by ply, exactly what hz_legal_mask + hz_rule_actions + hz_step write
    (mask, count, action, status), and leaves the same states and streams;
    the final states are the C oracle's games (1000 boards: a partial
    block; the env's second episode, so the reset counter is exercised)."""
    from hzamd.env import BatchedEnv
    n, base = 1000, 2024
    envs = [BatchedEnv(n, seed_base=base, device=DEV) for _ in range(2)]
    for e in envs:
        e.reset()
        e.reset()
    outs = [[torch.zeros(n, 3, dtype=torch.int64, device=DEV), torch.zeros(n, dtype=torch.int32, device=DEV),
             torch.zeros(n, dtype=torch.int16, device=DEV), torch.zeros(n, dtype=torch.int32, device=DEV)]
            for _ in range(2)]
    for p in range(96):
        m, c, a, s = outs[0]
        envs[0].legal_mask(m, c)
        envs[0].rule_actions(m, c, a)
        envs[0].step(a, s)
        envs[1].rule_ply(*outs[1])
        for x, y in zip(*outs):
            assert torch.equal(x, y), p
    st = [e.export_state(with_mt=True) for e in envs]
    for x, y in zip(*st):
        assert torch.equal(x, y)
    _, finals, plies, _ = oracle.play_rule_games(n, base, nthreads=8, episode=1)
    assert (states_of(envs[1]) == finals).all()
    assert bool(envs[1].done().all())
    for e in envs:
        e.close()


@pytest.mark.parametrize("plies", [96, 40, 250])
def test_auto_reset_prepared_episodes_equal_in_place_seeding(Env, plies):
    """hz_rollout(auto_reset) with episodes prepared ahead (the default) and
    with every new game seeded in place (hz_env_set_auto_ahead(0)): the same
    states, CPython streams (exported mid-run and at the end: boards then
    play on streams copied back from the preparation slots), game and step
    counts, on a partial block of boards; 250 plies per call ends up to four
    games per board per call (only the first two may come from the slots);
    and the final states and game counts equal the oracle's auto-reset
    restatement."""
    n, base, calls = 1000, 4242, 7
    outs = []
    for on in (True, False):
        env = Env(n, seed_base=base, device=DEV)
        env.set_auto_ahead(on)
        env.reset()
        games = torch.zeros(calls, n, dtype=torch.int32, device=DEV)
        steps = torch.zeros(calls, n, dtype=torch.int32, device=DEV)
        mid = None
        for c in range(calls):
            env.rollout(plies, auto_reset=True, games_done=games[c], steps_done=steps[c])
            if c == 3:
                mid = tuple(t.clone() for t in env.export_state(with_mt=True))
        fin = env.export_state(with_mt=True)
        env.check_errors()
        outs.append([t.cpu() for t in (*mid, *fin, games.sum(0), steps.sum(0))])
        env.close()
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    total, finals, ref_games, _ = oracle.play_rule_auto(n, base, calls * plies, ep0=0, nthreads=8)
    st = outs[0][3].numpy()
    g = outs[0][6].numpy()
    bad = [b for b in range(n) if not ((unpack_ref(st[:, b]) == finals[b]).all() and g[b] == ref_games[b])]
    assert not bad, bad[:8]
    assert int(outs[0][7].sum()) == total


def test_auto_reset_then_per_ply_steps_continue_the_streams(Env):
    """After auto-reset calls that left boards on prepared slots, the per-ply
    surface (hz_rule_ply) continues every board's game and stream exactly as
    after in-place seeding (the slots' streams materialised first)."""
    n, base = 700, 77
    outs = []
    for on in (True, False):
        env = Env(n, seed_base=base, device=DEV)
        env.set_auto_ahead(on)
        env.reset()
        for _ in range(5):
            env.rollout(96, auto_reset=True)
        for _ in range(30):
            env.rule_ply()
        outs.append([t.cpu() for t in env.export_state(with_mt=True)])
        env.close()
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("fused", [True, False])
def test_ply_window_slots_never_change_results(Env, fused):
    """hz_rule_ply / hz_step keep 12 stream words per board from the ply
    before a turn end (PlyWin, tagged with the cursor and the stream epoch
    that every stream-rewriting entry point bumps).  Boards whose streams are
    replaced mid-turn by hz_import_state at the same CPython index, then
    played on, match a fresh env given the same states and streams: every
    state and stream after 12 more plies; and a run that crosses turn ends
    uninterrupted matches the oracle's rule games."""
    n = 300

    def ply(env):
        if fused:
            env.rule_ply()
        else:
            mask, count = env.legal_mask()
            env.step(env.rule_actions(mask, count))

    a = Env(n, seed_base=5, device=DEV)
    a.reset()
    for _ in range(7):  # plies 0-6: windows saved after plies 2 and 6 (turn ends at 3, 7)
        ply(a)
    st, _, idx = a.export_state(with_mt=True)
    other = Env(n, seed_base=91, device=DEV)
    other.reset()
    _, mt2, _ = other.export_state(with_mt=True)
    a.import_state(st, mt2, idx)  # other words at the same cursors
    for _ in range(12):
        ply(a)
    got = states_of(a)
    _, mt, mi = a.export_state(with_mt=True)
    mt, mi = mt.cpu().numpy().view(np.uint32), mi.cpu().numpy()
    st, mt2, idx = st.cpu().numpy(), mt2.cpu().numpy().view(np.uint32), idx.cpu().numpy()
    for b in range(0, n, 7):  # the oracle from the imported state and stream (rule seed 5 + b, ply 7)
        s = unpack_ref(st[:, b])
        m = oracle.mt_from_words(mt2[b], idx[b])
        for p in range(7, 19):
            if oracle.is_game_over(s):
                break
            mask = oracle.legal(s)
            L = int(mask.sum())
            act = np.flatnonzero(mask)[((oracle.rule(5 + b, p) >> 32) * L) >> 32]
            s = oracle.step(s, int(act), m)[1]
        assert (got[b] == s).all(), b
        assert oracle.mt_next32(oracle.mt_from_words(mt[b], mi[b])) == oracle.mt_next32(m), b
    # uninterrupted: whole rule games, turn ends drawing from saved words
    d = Env(n, seed_base=17, device=DEV)
    d.reset()
    for _ in range(96):
        ply(d)
    _, finals, _, nxt = oracle.play_rule_games(n, 17, nthreads=8)
    got = states_of(d)
    _, mt, mi = d.export_state(with_mt=True)
    mt, mi = mt.cpu().numpy().view(np.uint32), mi.cpu().numpy()
    for b in range(n):
        assert (got[b] == finals[b]).all(), b
        assert oracle.mt_next32(oracle.mt_from_words(mt[b], mi[b])) == nxt[b], b


def test_legal_actions_bytes_equal_unpacked_mask(Env):
    """hz_legal_actions (BatchedEnv.legal_actions: one byte per action, one
    launch) equals the packed hz_legal_mask unpacked bit by bit, counts
    included, on a partial block of boards spread over the game (finished
    boards: all false)."""
    from hzamd.env import unpack_mask
    n = 1000
    env = Env(n, seed_base=303, device=DEV)
    env.reset()
    plies = torch.arange(n, device=DEV) % 75
    for p in range(75):
        mask, count = env.legal_mask()
        act = env.rule_actions(mask, count)
        env.step(torch.where(plies > p, act, torch.full_like(act, -1)))
    mask, count = env.legal_mask()
    want, want_c = unpack_mask(mask).clone(), count.clone()
    got = env.legal_actions()
    assert got.dtype == torch.bool and got.shape == (n, 143)
    assert torch.equal(got, want) and torch.equal(env._count, want_c)
    assert bool((got.sum(1) == want_c).all()) and bool((want_c == 0).any())


@pytest.mark.gpu
def test_caller_buffers_are_checked_before_launch(Env):
    """A caller-supplied output buffer of the wrong shape, dtype or device is
    refused with ValueError before its pointer reaches the library (the
    kernels write n rows whatever the buffer holds); correct ones are used."""
    n = 130
    env = Env(n, seed_base=5, device=DEV)
    env.reset()
    bad = [
        lambda: env.legal_actions(out=torch.zeros(n - 1, 143, dtype=torch.bool, device=DEV)),
        lambda: env.legal_actions(out=torch.zeros(n, 143, dtype=torch.uint8, device=DEV)),
        lambda: env.legal_actions(out=torch.zeros(n, 2 * 143, dtype=torch.bool, device=DEV)[:, ::2]),
        lambda: env.legal_mask(out=torch.zeros(n, 3, dtype=torch.int64)),
        lambda: env.legal_mask(count=torch.zeros(n, dtype=torch.int64, device=DEV)),
        lambda: env.step(torch.zeros(n, dtype=torch.int16, device=DEV), status=torch.zeros(n - 2, dtype=torch.int32,
                                                                                            device=DEV)),
        lambda: env.rule_ply(torch.zeros(n, 2, dtype=torch.int64, device=DEV)),
        lambda: env.rollout(4, games_done=torch.zeros(n // 2, dtype=torch.int32, device=DEV)),
    ]
    for f in bad:
        with pytest.raises(ValueError):
            f()
    out = torch.ones(n, 143, dtype=torch.bool, device=DEV)
    assert env.legal_actions(out=out) is out and int(out.sum()) == int(env._count.sum()) > 0


@pytest.mark.gpu
def test_large_ragged_batch_vs_oracle(Env):
    """16x the BASELINE batch plus a ragged tail (65,573 boards: 1,025 blocks
    of 64, the last with 37 boards; many rounds of blocks per launch): the
    thirteen-stage hz_play pipeline once full (episodes 12, 13), the
    auto-reset rollout and the per-ply hz_rule_ply path, every board's final
    state, ply / step counts and a sample of streams bit-exact vs the C
    oracle."""
    n, base = 65_573, 90_001
    env = Env(n, seed_base=base, device=DEV)
    env.set_pipeline(2)
    for ep in range(14):
        _, steps, _ = env.rollout(200, reset=True)
        if ep >= 12:
            total, finals, plies, nxt = oracle.play_rule_games(n, base, nthreads=8, episode=ep)
            assert (states_of(env) == finals).all(), ep
            assert (steps.cpu().numpy() == plies).all() and int(steps.sum()) == total, ep
            _, mt, idx = env.export_state(with_mt=True)
            mt, idx = mt.cpu().numpy().view(np.uint32), idx.cpu().numpy()
            for b in list(range(0, n, 4099)) + [n - 1]:
                assert oracle.mt_next32(oracle.mt_from_words(mt[b], idx[b])) == nxt[b], (ep, b)
    env.check_errors()
    env.close()

    env = Env(n, seed_base=base, device=DEV)
    env.reset()
    games, steps, _ = env.rollout(96, auto_reset=True)
    total, finals, g_want, ep_want = oracle.play_rule_auto(n, base, 96, ep0=0, nthreads=8)
    assert int(steps.sum()) == total and (games.cpu().numpy() == g_want).all()
    assert (states_of(env) == finals).all()
    env.close()

    env = Env(n, seed_base=base, device=DEV)
    env.reset()
    for _ in range(96):
        env.rule_ply()
    total, finals, plies, _ = oracle.play_rule_games(n, base, nthreads=8, episode=0)
    assert (states_of(env) == finals).all()
    env.close()


@pytest.mark.gpu
def test_single_board_every_path(Env):
    """One board (a block with 63 idle lanes in every role): the thirteen-stage
    hz_play until fully pipelined, the chance-ahead pipeline, the auto-reset
    rollout, the per-ply surface and the byte mask, each bit-exact vs the
    oracle."""
    n, base = 1, 61
    env = Env(n, seed_base=base, device=DEV)
    env.set_pipeline(2)
    for ep in range(15):
        _, steps, _ = env.rollout(200, reset=True)
        _check_episode(env, base, ep, steps)
    env.set_pipeline(1)
    for ep in range(15, 19):
        _, steps, _ = env.rollout(200, reset=True)
        _check_episode(env, base, ep, steps)
    env.check_errors()
    env.close()

    env = Env(n, seed_base=base, device=DEV)
    env.reset()
    games, steps, _ = env.rollout(300, auto_reset=True)
    total, finals, g_want, _ = oracle.play_rule_auto(n, base, 300, ep0=0, nthreads=1)
    assert int(steps.sum()) == total and (games.cpu().numpy() == g_want).all()
    assert (states_of(env) == finals).all()
    env.close()

    env = Env(n, seed_base=base, device=DEV)
    env.reset()
    while not bool(env.done().all()):
        legal = env.legal_actions()
        mask, count = env.legal_mask()
        from hzamd.env import unpack_mask
        assert torch.equal(legal, unpack_mask(mask)) and int(legal.sum()) == int(count[0])
        env.rule_ply()
    total, finals, plies, _ = oracle.play_rule_games(n, base, nthreads=1, episode=0)
    assert (states_of(env) == finals).all()
    env.close()
