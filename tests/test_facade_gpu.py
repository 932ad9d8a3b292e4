"""The drop-in modules (harmonies_engine / process_game_state / MCTS in
harmonies-alphazero_amd/) behave like the reference modules: the reference's
own engine tests (tests/test_harmonies_engine.py: immutability of apply_move,
hash/eq semantics) restated, seeded games equal the golden traces (including
the global `random` stream), encoder outputs equal the golden tensors, and
get_best_action_and_pi reproduces the golden searches."""
import os
import random

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def load(name):
    return np.load(os.path.join(GOLDEN, name))


@pytest.fixture(scope="module")
def he():
    import harmonies_engine
    return harmonies_engine


# ---- restatement of the reference unit tests (test_harmonies_engine.py) ----

def test_apply_move_returns_new_object_and_leaves_original(he):
    random.seed(11)
    s = he.HarmoniesGameState()
    snap = s.clone()
    t = s.apply_move(0)
    assert t is not s
    assert s.current_player == snap.current_player and s.turn_phase == snap.turn_phase
    assert s.tiles_in_hand == snap.tiles_in_hand and len(s.available_piles) == len(snap.available_piles)


def test_choose_pile_updates_phase_hand_and_piles(he):
    random.seed(12)
    s = he.HarmoniesGameState()
    pile = list(s.available_piles[0])
    n = len(s.available_piles)
    t = s.apply_move(0)
    assert t.turn_phase == "place_tile_1" and s.turn_phase == "choose_pile" and s.current_player == 0
    assert len(t.available_piles) == n - 1 and len(t.tiles_in_hand) == he.PILE_SIZE
    assert sorted(t.tiles_in_hand) == sorted(pile)
    assert len(s.available_piles) == n and s.tiles_in_hand == []
    assert t.tile_bag == s.tile_bag and t.player_boards == s.player_boards


def test_hash_and_eq_follow_canonical_tuple(he):
    random.seed(13)
    a = he.HarmoniesGameState()
    a.available_piles = [["a", "b", "c"], ["d", "e", "f"]]
    a.tile_bag = {"a": 1, "b": 1, "c": 1}
    b = a.clone()
    assert a == b and hash(a) == hash(b)
    for field, value in [("current_player", 1), ("turn_phase", "place_tile_1"), ("tiles_in_hand", ["a", "c"]),
                         ("available_piles", [["a", "b", "c"], ["X", "Y", "Z"]]), ("tile_bag", {"a": 2, "b": 1, "c": 1}),
                         ("player_boards", [{(1, 0): ["a"]}, {}])]:
        c = a.clone()
        setattr(c, field, value)
        assert c != a and hash(c) != hash(a), field


# ---- seeded games through the facade equal the reference traces -----------

def test_seeded_games_match_traces(he):
    from hzamd.state import ref_from_object
    import process_game_state as pgs
    f = load("env_traces.npz")
    off = f["offsets"]
    for g in range(0, 64, 8):
        seed = int(f["seeds"][g])
        random.seed(seed)
        s = he.HarmoniesGameState()
        for ply in range(off[g + 1] - off[g]):
            p = off[g] + ply
            assert (ref_from_object(s) == f["states"][p]).all(), (g, ply)
            moves = s.get_legal_moves()
            idx = [pgs.get_action_index(m) for m in moves]
            assert idx == sorted(idx)
            mask = np.zeros(143, np.uint8)
            mask[idx] = 1
            assert (np.packbits(mask, bitorder="little") == f["masks"][p]).all()
            x = oracle_rule(seed, ply, len(moves))
            assert pgs.get_action_index(moves[x]) == f["actions"][p]
            s = s.apply_move(moves[x])
        assert (ref_from_object(s) == f["finals"][g]).all()
        assert s.is_game_over()
        assert random.getrandbits(32) == f["next_word"][g]
        assert s.get_game_outcome() in (1, -1, 0)
        assert s.calculate_score_for_player(0) == s.final_scores[0]


def oracle_rule(seed, ply, L):
    import oracle
    return int(((oracle.rule(seed, ply) >> 32) * L) >> 32)


def test_apply_move_errors_match_reference_messages(he):
    random.seed(5)
    s = he.HarmoniesGameState()
    with pytest.raises(ValueError, match="Invalid pile index"):
        s.apply_move(9)
    with pytest.raises(ValueError, match="Invalid pile index"):
        s.apply_move(("water", (0, 0)))
    t = s.apply_move(0)
    with pytest.raises(ValueError, match="Invalid move format"):
        t.apply_move(0)
    with pytest.raises(ValueError, match="Invalid coordinate"):
        t.apply_move(("water", (9, 9)))
    missing = [x for x in he.TILE_TYPES if x not in t.tiles_in_hand][0]
    with pytest.raises(ValueError, match="not found in hand"):
        t.apply_move((missing, (0, 0)))
    over = t.clone()
    over.turn_phase = "game_over"
    with pytest.raises(ValueError, match="Invalid turn phase"):
        over.apply_move(0)


def test_end_turn_and_scoring_helpers(he):
    f = load("scoring.npz")
    from hzamd.state import SORTED_COORDS, STACKS
    g = he.HarmoniesGameState.__new__(he.HarmoniesGameState)
    for b, sc in zip(f["boards"][:40], f["scores"][:40]):
        board = {SORTED_COORDS[c]: list(STACKS[int(b[c])]) for c in range(23) if b[c]}
        got = [g._score_grass(board, 0), g._score_mountains(board, 0), g._score_fields(board, 0),
               g._score_buildings(board, 0), g._score_water(board, 0)]
        assert got == list(sc)
    assert he.get_water_score(1) == 0 and he.get_water_score(6) == 15 and he.get_water_score(8) == 23
    assert sorted(he.get_neighbors((0, 0))) == sorted([(1, 0), (-1, 0), (0, 1), (0, -1), (1, -1), (-1, 1)])


def test_create_state_tensors_matches_reference(he):
    import process_game_state as pgs
    from hzamd.state import apply_ref_to_object
    f = load("encoder.npz")
    for st, b, g in list(zip(f["states"], f["boards"], f["globs"]))[::16]:
        obj = apply_ref_to_object(st, he.HarmoniesGameState.__new__(he.HarmoniesGameState))
        tb, tg = pgs.create_state_tensors(obj)
        assert tb.dtype == torch.float32 and tb.shape == (38, 5, 7) and tb.device.type == "cpu"
        assert (tb.numpy() == b).all() and (tg.numpy() == g).all()


class _StubManager:
    def predict(self, board, glob):
        import oracle
        from hzamd.mcts import stub_evaluator
        p, v = stub_evaluator(board.unsqueeze(0), glob.unsqueeze(0))
        return p[0].numpy(), float(v[0])


def test_get_best_action_and_pi_matches_golden(he):
    import MCTS
    import process_game_state as pgs
    from hzamd.state import apply_ref_to_object
    f = load("mcts.npz")
    for k in range(0, 80, 5):
        sims = int(f["sims"][k])
        obj = apply_ref_to_object(f["state"][k], he.HarmoniesGameState.__new__(he.HarmoniesGameState))
        cfg = {"num_simulations": sims, "cpuct": float(f["cpuct"][k]), "dirichlet_alpha": 0.4,
               "dirichlet_epsilon": float(f["eps"][k]), "turns_until_tau0": int(f["tau0"][k]),
               "action_size": 143, "testing": bool(f["testing"][k])}
        noise = f["noise"][k]
        u = float(f["u"][k])

        def fake_dirichlet(alpha):
            return noise[:len(alpha)].copy()

        def fake_choice(n, p):
            T = sims - 1
            c = np.rint(np.asarray(p) * T).astype(np.int64)
            return int(np.argmax(u * T < np.cumsum(c)))

        saved = (np.random.dirichlet, np.random.choice)
        np.random.dirichlet, np.random.choice = fake_dirichlet, fake_choice
        try:
            random.seed(int(f["mt_seed"][k]))
            mv, pi = MCTS.get_best_action_and_pi(obj, _StubManager(), cfg, int(f["ply"][k]))
            nxt = random.getrandbits(32)
        finally:
            np.random.dirichlet, np.random.choice = saved
        assert np.allclose(pi, f["pi"][k], rtol=0, atol=0), k
        assert pgs.get_action_index(mv) == f["action"][k], k
        assert nxt == f["next_word"][k], k


def test_get_best_action_and_pi_with_model_manager_device_rows(he):
    """With hzamd's ModelManager the drop-in search evaluates its leaves on
    the device (the folded network that predict() runs, no host round trip
    per simulation); any other manager goes through predict().  Both give
    the same move, pi and Python RNG state on the same positions."""
    import MCTS
    from hzamd.manager import ModelManager
    from hzamd.net import DEFAULT
    from hzamd.state import apply_ref_to_object
    from test_manager_cpu import TRAIN_CFG
    torch.manual_seed(0)
    mm = ModelManager(dict(DEFAULT), dict(TRAIN_CFG, device="cuda:0"))

    class ViaPredict:  # no _fast: MCTS uses predict() per leaf
        def predict(self, board, glob):
            return mm.predict(board, glob)

    f = load("mcts.npz")
    cfg = {"num_simulations": 24, "cpuct": 2.0, "dirichlet_alpha": 0.4, "dirichlet_epsilon": 0.25,
           "turns_until_tau0": 15, "action_size": 143, "testing": True}
    for k in range(0, 80, 10):
        out = []
        for manager in (mm, ViaPredict()):
            obj = apply_ref_to_object(f["state"][k], he.HarmoniesGameState.__new__(he.HarmoniesGameState))
            random.seed(int(f["mt_seed"][k]))
            mv, pi = MCTS.get_best_action_and_pi(obj, manager, cfg, 20)
            out.append((mv, pi, random.getrandbits(32)))
        assert isinstance(MCTS._evaluator(mm, "cuda:0"), MCTS._FoldedRows)
        (m0, p0, r0), (m1, p1, r1) = out
        assert m0 == m1 and np.array_equal(p0, p1) and r0 == r1, k


def test_get_best_action_and_pi_graph_cache(he):
    """The drop-in search replays one captured simulation (HIP graph) kept
    across moves; the result equals the eager search on the same positions,
    with noise and sampling (testing=False), and after a weight change (the
    network's generation changes: the kept graph is not reused)."""
    import MCTS
    from hzamd.manager import ModelManager
    from hzamd.net import DEFAULT
    from hzamd.state import apply_ref_to_object
    from test_manager_cpu import TRAIN_CFG
    torch.manual_seed(1)
    mm = ModelManager(dict(DEFAULT), dict(TRAIN_CFG, device="cuda:0"))
    f = load("mcts.npz")
    cfg = {"num_simulations": 16, "cpuct": 2.0, "dirichlet_alpha": 0.4, "dirichlet_epsilon": 0.25,
           "turns_until_tau0": 15, "action_size": 143, "testing": False}

    def run(k, graph):
        MCTS.GRAPH = graph
        try:
            obj = apply_ref_to_object(f["state"][k], he.HarmoniesGameState.__new__(he.HarmoniesGameState))
            random.seed(int(f["mt_seed"][k]))
            np.random.seed(k)
            mv, pi = MCTS.get_best_action_and_pi(obj, mm, cfg, 3)
            return mv, pi, random.getrandbits(32)
        finally:
            MCTS.GRAPH = True

    for phase in range(2):
        for k in range(0, 80, 16):
            (m0, p0, r0), (m1, p1, r1) = run(k, True), run(k, False)
            assert m0 == m1 and np.array_equal(p0, p1) and r0 == r1, (phase, k)
        gen = mm._fast().generation
        with torch.no_grad():
            for prm in mm.model.parameters():
                prm.mul_(1.5)
        assert mm._fast().generation == gen + 1
