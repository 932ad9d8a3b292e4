"""Golden-vector capture from the reference engine (TEST INFRASTRUCTURE).

Runs ONLY in the build container, where the reference checkout is mounted at
/root/reference.  It imports the reference's own Python modules (behind a
`loggers` shim: reference loggers.py:22-35 opens FileHandlers under a
read-only directory) and writes small .npz fixtures next to this file.  The
tests read only those .npz files; nothing here travels to the GPU box or is
imported by the product.

Fixtures (all int arrays unless noted; REFSTATE = 78 x int16, see `ref_state`):
  mt_streams.npz     CPython MT19937 outputs (random.seed(int) + getrandbits(32))
                     and random.sample(range(n), 3) results.
  env_traces.npz     per-ply REFSTATE + 143-bit legal mask + action for seeded
                     games driven by the build-defined splitmix rule (never
                     touches `random`), plus final scores/winner/next MT word.
  env_finals.npz     final REFSTATE for 1024 more seeds.
  encoder.npz        create_state_tensors() outputs (f32) at sampled states.
  scoring.npz        per-habitat scores of the known-answer board
                     and of random reachable-stack boards.
  greedy.npz         greedy-vs-greedy games of evaluation.choose_move_greedy
                     (canonical move order): per-ply REFSTATE + chosen action,
                     final state and next MT word (the greedy agent's
                     simulated apply_move calls consume `random` too).
  train.npz          ModelManager.train_step (model.py:112-157) on the test
                     model config: initial / final state_dict, batch, losses;
  ref_ckpt_tiny.pth.tar  the same manager's save_checkpoint (model.py:159-182)
                     output after those steps (iteration 7), for the loader.
  mcts.npz           get_best_action_and_pi() root visit counts, chosen move,
                     tree size and next MT word under a canonical (ascending
                     action index) move order and a deterministic stub
                     evaluator; testing=True and testing=False (noise/choice
                     injected through patched numpy calls).

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [part ...]
        (parts: mt env encoder scoring mcts greedy train; default all)
"""
import logging
import os
import random
import sys
import types

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
M64 = (1 << 64) - 1

TILES = ["water", "plant", "wood", "stone", "building", "field"]
PHASES = ["choose_pile", "place_tile_1", "place_tile_2", "place_tile_3", "game_over"]
# Stack codes: every stack the placement rules can build
# (reference harmonies_engine.py:183-194 / :254-283).
CODES = [
    (),
    ("water",), ("plant",), ("wood",), ("stone",), ("building",), ("field",),
    ("wood", "plant"), ("stone", "stone"), ("stone", "stone", "stone"),
    ("wood", "building"), ("stone", "building"), ("building", "building"),
]
CODE_OF = {c: i for i, c in enumerate(CODES)}
INITIAL_TT = [23, 19, 21, 23, 15, 19]  # INITIAL_BAG in TILE_TYPES order


def import_reference():
    shim = types.ModuleType("loggers")
    for name in ["logger_mcts", "logger_main", "logger_tourney", "logger_memory", "logger_model"]:
        lg = logging.getLogger("golden_" + name)
        lg.addHandler(logging.NullHandler())
        lg.propagate = False
        setattr(shim, name, lg)
    sys.modules["loggers"] = shim
    sys.path.insert(0, REF)
    import harmonies_engine as he  # noqa: E402
    import process_game_state as pgs  # noqa: E402
    import MCTS as mcts_mod  # noqa: E402
    return he, pgs, mcts_mod


def splitmix_rule(seed, ply):
    """Build-defined deterministic action rule (does not touch `random`)."""
    x = (seed * 0x9E3779B97F4A7C15 + ply) & M64
    z = (x + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def pick_index(seed, ply, n_legal):
    z = splitmix_rule(seed, ply)
    return ((z >> 32) * n_legal) >> 32


def ref_state(g, idx_of):
    v = np.zeros(78, np.int16)
    for p in (0, 1):
        for coord, stack in g.player_boards[p].items():
            v[p * 23 + idx_of[coord]] = CODE_OF[tuple(stack)]
    v[46:61] = -1
    for i, pile in enumerate(g.available_piles):
        for j, t in enumerate(pile):
            v[46 + i * 3 + j] = TILES.index(t)
    v[61] = len(g.available_piles)
    v[62:65] = -1
    for j, t in enumerate(g.tiles_in_hand):
        v[62 + j] = TILES.index(t)
    v[65] = len(g.tiles_in_hand)
    assert list(g.tile_bag.keys()) == ["water", "plant", "wood", "stone", "field", "building"]
    for t, name in enumerate(TILES):
        v[66 + t] = g.tile_bag[name]
    v[72] = g.current_player
    v[73] = PHASES.index(g.turn_phase)
    v[74] = int(bool(g.game_over))
    v[75] = -2 if g.winner is None else g.winner
    v[76] = g.final_scores[0]
    v[77] = g.final_scores[1]
    return v


def legal_sorted(g, pgs, orig_get_legal):
    return sorted(orig_get_legal(g), key=pgs.get_action_index)


def mask_bits(moves, pgs):
    m = np.zeros(143, np.uint8)
    for mv in moves:
        m[pgs.get_action_index(mv)] = 1
    return np.packbits(m, bitorder="little")  # 18 bytes


def capture_mt():
    seeds = [0, 1, 12345, (1 << 40) + 7, 2**32 - 1, 2**32]
    words = np.zeros((len(seeds), 1000), np.uint32)
    for i, s in enumerate(seeds):
        random.seed(s)
        for k in range(1000):
            words[i, k] = random.getrandbits(32)
    ns = np.arange(3, 121, 3)
    samp = np.zeros((len(seeds), len(ns), 3), np.int32)
    nxt = np.zeros((len(seeds),), np.uint32)
    for i, s in enumerate(seeds):
        random.seed(s)
        for j, n in enumerate(ns):
            samp[i, j] = random.sample(range(int(n)), 3)
        nxt[i] = random.getrandbits(32)
    # small populations exercise the pool path (n <= 21) incl. k = n < 3
    small = np.full((len(seeds), 21, 3), -1, np.int32)
    for i, s in enumerate(seeds):
        random.seed(s)
        for n in range(1, 22):
            k = min(3, n)
            small[i, n - 1, :k] = random.sample(range(n), k)
    np.savez_compressed(os.path.join(OUT, "mt_streams.npz"), seeds=np.array(seeds, np.uint64),
                        words=words, sample_n=ns.astype(np.int32), sample=samp, next_word=nxt,
                        small_sample=small)


def play_game(he, pgs, orig_get_legal, seed, idx_of, record):
    random.seed(seed)
    g = he.HarmoniesGameState()
    states, masks, acts = [], [], []
    ply = 0
    while not g.is_game_over():
        moves = legal_sorted(g, pgs, orig_get_legal)
        assert moves, "stuck board"
        k = pick_index(seed, ply, len(moves))
        mv = moves[k]
        if record:
            states.append(ref_state(g, idx_of))
            masks.append(mask_bits(moves, pgs))
            acts.append(pgs.get_action_index(mv))
        g = g.apply_move(mv)
        ply += 1
    final = ref_state(g, idx_of)
    return g, ply, states, masks, acts, final, random.getrandbits(32)


def capture_env(he, pgs, idx_of):
    orig = he.HarmoniesGameState.get_legal_moves
    st, mk, ac, off, fin, plies, nxt, seeds = [], [], [], [0], [], [], [], list(range(64))
    for s in seeds:
        g, ply, states, masks, acts, final, nw = play_game(he, pgs, orig, s, idx_of, True)
        st += states; mk += masks; ac += acts
        off.append(off[-1] + len(states))
        fin.append(final); plies.append(ply); nxt.append(nw)
    np.savez_compressed(os.path.join(OUT, "env_traces.npz"), seeds=np.array(seeds, np.uint64),
                        states=np.array(st, np.int16), masks=np.array(mk, np.uint8),
                        actions=np.array(ac, np.int16), offsets=np.array(off, np.int32),
                        finals=np.array(fin, np.int16), plies=np.array(plies, np.int32),
                        next_word=np.array(nxt, np.uint32))
    fseeds = list(range(1000, 2024))
    fin, plies, nxt = [], [], []
    for s in fseeds:
        g, ply, _, _, _, final, nw = play_game(he, pgs, orig, s, idx_of, False)
        fin.append(final); plies.append(ply); nxt.append(nw)
    np.savez_compressed(os.path.join(OUT, "env_finals.npz"), seeds=np.array(fseeds, np.uint64),
                        finals=np.array(fin, np.int16), plies=np.array(plies, np.int32),
                        next_word=np.array(nxt, np.uint32))
    return np.array(st, np.int16)


def state_from_ref(he, v, sorted_coords):
    g = he.HarmoniesGameState.__new__(he.HarmoniesGameState)
    g.player_boards = [{}, {}]
    for p in (0, 1):
        for c in range(23):
            code = int(v[p * 23 + c])
            if code:
                g.player_boards[p][sorted_coords[c]] = list(CODES[code])
    g.tile_bag = {}
    for name in ["water", "plant", "wood", "stone", "field", "building"]:
        g.tile_bag[name] = int(v[66 + TILES.index(name)])
    g.available_piles = []
    for i in range(int(v[61])):
        g.available_piles.append([TILES[int(t)] for t in v[46 + 3 * i: 49 + 3 * i] if t >= 0])
    g.tiles_in_hand = [TILES[int(t)] for t in v[62:62 + int(v[65])]]
    g.current_player = int(v[72])
    g.turn_phase = PHASES[int(v[73])]
    g.game_over = bool(v[74])
    g.winner = None if v[75] == -2 else int(v[75])
    g.final_scores = [int(v[76]), int(v[77])]
    return g


def capture_encoder(he, pgs, states, sorted_coords, idx_of):
    rng = np.random.RandomState(7)
    pick = rng.choice(len(states), 256, replace=False)
    sel = states[np.sort(pick)]
    boards, globs = [], []
    for v in sel:
        g = state_from_ref(he, v, sorted_coords)
        assert (ref_state(g, idx_of) == v).all()
        b, gl = pgs.create_state_tensors(g)
        boards.append(b.numpy()); globs.append(gl.numpy())
    # plus game_over-phase states (channel 37 = 0) from the finals
    np.savez_compressed(os.path.join(OUT, "encoder.npz"), states=sel,
                        boards=np.array(boards, np.float32), globs=np.array(globs, np.float32))


def capture_scoring(he, sorted_coords, idx_of):
    g = he.HarmoniesGameState.__new__(he.HarmoniesGameState)
    fns = [g._score_grass, g._score_mountains, g._score_fields, g._score_buildings, g._score_water]
    known = {(0, 0): ["water"], (1, 0): ["water"], (2, 0): ["water"], (0, 1): ["field"],
             (1, 1): ["field"], (-1, 0): ["stone", "stone"], (-1, 1): ["stone"],
             (2, -1): ["wood", "building"], (2, -2): ["wood", "plant"],
             (1, -1): ["stone", "stone", "stone"], (3, -2): ["plant"]}
    boards = []
    b = np.zeros(23, np.uint8)
    for coord, st in known.items():
        b[idx_of[coord]] = CODE_OF[tuple(st)]
    boards.append(b)
    rng = np.random.RandomState(11)
    for i in range(4000):
        fill = rng.uniform(0.2, 1.0)
        # bias towards water/field/stone-heavy boards every few samples
        if i % 4 == 0:
            probs = np.array([0, 6, 1, 1, 2, 1, 5, 1, 1, 1, 1, 1, 1], float)
        elif i % 4 == 1:
            probs = np.array([0, 1, 1, 1, 5, 1, 1, 1, 3, 3, 1, 1, 1], float)
        else:
            probs = np.array([0] + [1] * 12, float)
        probs /= probs.sum()
        b = np.where(rng.uniform(size=23) < fill, rng.choice(13, size=23, p=probs), 0).astype(np.uint8)
        boards.append(b)
    scores = np.zeros((len(boards), 5), np.int32)
    for k, b in enumerate(boards):
        board = {sorted_coords[c]: list(CODES[int(b[c])]) for c in range(23) if b[c]}
        for j, f in enumerate(fns):
            scores[k, j] = f(board, 0)
    assert list(scores[0]) == [4, 4, 5, 5, 5], scores[0]
    np.savez_compressed(os.path.join(OUT, "scoring.npz"), boards=np.array(boards, np.uint8), scores=scores)


# ---- MCTS -------------------------------------------------------------------

def stub_predict_np(board, glob):
    """Deterministic stub evaluator; integer arithmetic only so that a torch
    restatement on the GPU produces bit-identical priors/values."""
    b = np.asarray(board, np.float32)
    gl = np.asarray(glob, np.float32)
    n0 = int(np.rint(b[0:18].sum(dtype=np.float64)))
    n1 = int(np.rint(b[18:36].sum(dtype=np.float64)))
    cp = int(np.rint(b[36].max()))
    ph3 = int(np.rint(b[37].max() * 3.0))
    pc = np.rint(gl[0:36].astype(np.float64) * 3.0).astype(np.int64)
    w = int((pc * np.arange(1, 37, dtype=np.int64)).sum())
    K = (n0 * 73 + n1 * 151 + ph3 * 7 + cp * 3 + w * 13) % (1 << 31)
    a = np.arange(143, dtype=np.int64)
    h = (a * 2654435761 + K * 40503) % (1 << 32)
    pol = ((h >> 22) + 1).astype(np.float32) / np.float32(1024.0)
    val = float(((K % 255) - 127) / 128.0)
    return pol, val


class StubManager:
    def predict(self, board, glob):
        return stub_predict_np(board.numpy(), glob.numpy())


def capture_mcts(he, pgs, mcts_mod, states, sorted_coords, idx_of):
    orig = he.HarmoniesGameState.get_legal_moves
    he.HarmoniesGameState.get_legal_moves = lambda self: sorted(orig(self), key=pgs.get_action_index)
    last = {}
    orig_init = mcts_mod.MCTS.__init__

    def init(self, root, cfg):
        orig_init(self, root, cfg)
        last["tree"] = self
    mcts_mod.MCTS.__init__ = init

    rng = np.random.RandomState(3)
    # positions: states from the traces, biased to include late-game ones
    n = len(states)
    idx = list(rng.choice(n, 56, replace=False))
    late = [i for i in range(n) if states[i][73] != 4 and (23 - (states[i][0:23] > 0).sum()) <= 4]
    idx += list(rng.choice(late, 24, replace=False))
    rows = []
    for k, si in enumerate(idx):
        v = states[si]
        testing = (k % 3) != 2
        sims = [32, 8, 64, 200][k % 4] if k < 76 else 400
        cpuct = [2, 1.0, 2, 1.5][k % 4]
        mt_seed = 5000 + k
        noise = np.zeros(143, np.float64)
        u = ((k * 0.6180339887498949) % 1.0)
        cfg = {"num_simulations": sims, "cpuct": cpuct, "dirichlet_alpha": 0.4,
               "dirichlet_epsilon": 0.25 if k % 6 != 5 else 0, "fpu_value": 0.25,
               "turns_until_tau0": 15 if k % 5 else 0, "action_size": 143, "testing": testing}
        ply = k % 30
        choice_used = [False]

        def fake_dirichlet(alpha):
            L = len(alpha)
            raw = np.array([((j * 7 + k * 3) % 11 + 1) for j in range(L)], np.float64)
            vec = raw / raw.sum()
            noise[:L] = vec
            return vec

        def fake_choice(nact, p):
            choice_used[0] = True
            p = np.asarray(p, np.float64)
            T = sims - 1
            c = np.rint(p * T).astype(np.int64)
            assert c.sum() == T
            cum = np.cumsum(c)
            return int(np.argmax(u * T < cum))

        saved = (np.random.dirichlet, np.random.choice)
        np.random.dirichlet, np.random.choice = fake_dirichlet, fake_choice
        try:
            g = state_from_ref(he, v, sorted_coords)
            random.seed(mt_seed)
            mv, pi = mcts_mod.get_best_action_and_pi(g, StubManager(), cfg, ply)
            nxt = random.getrandbits(32)
        finally:
            np.random.dirichlet, np.random.choice = saved
        tree = last["tree"]
        n_edges = sum(len(nd.edges) for nd in tree.tree.values())
        root_edges = tree.root.edges
        visits = np.zeros(143, np.int32)
        for a, e in root_edges.items():
            visits[pgs.get_action_index(a)] = e.stats["N"]
        rows.append(dict(state=v, mt_seed=mt_seed, sims=sims, cpuct=float(cpuct),
                         eps=float(cfg["dirichlet_epsilon"]), alpha=0.4, testing=int(testing),
                         tau0=cfg["turns_until_tau0"], ply=ply, u=u, noise=noise.copy(),
                         visits=visits, pi=np.asarray(pi, np.float64),
                         action=pgs.get_action_index(mv), next_word=nxt,
                         n_nodes=len(tree.tree), n_edges=n_edges, sampled=int(choice_used[0])))
    he.HarmoniesGameState.get_legal_moves = orig
    mcts_mod.MCTS.__init__ = orig_init
    out = {key: np.array([r[key] for r in rows]) for key in rows[0]}
    np.savez_compressed(os.path.join(OUT, "mcts.npz"), **out)


def capture_greedy(he, pgs, idx_of, seeds=range(5000, 5032)):
    """Greedy (P0) vs greedy (P1) through evaluation.play_game's loop
    (evaluation.py:68-133) with evaluation.choose_move_greedy (:137-196)."""
    import evaluation as ev
    orig = he.HarmoniesGameState.get_legal_moves
    he.HarmoniesGameState.get_legal_moves = lambda self: sorted(orig(self), key=pgs.get_action_index)
    st, ac, off, fin, nxt = [], [], [0], [], []
    try:
        for seed in seeds:
            random.seed(seed)
            g = he.HarmoniesGameState()
            while not g.is_game_over():
                mv, _ = ev.choose_move_greedy(g.clone())
                st.append(ref_state(g, idx_of))
                ac.append(pgs.get_action_index(mv))
                g = g.apply_move(mv)
            off.append(len(st))
            fin.append(ref_state(g, idx_of))
            nxt.append(random.getrandbits(32))
    finally:
        he.HarmoniesGameState.get_legal_moves = orig
    np.savez_compressed(os.path.join(OUT, "greedy.npz"), seeds=np.array(list(seeds), np.uint64),
                        states=np.array(st, np.int16), actions=np.array(ac, np.int16),
                        offsets=np.array(off, np.int32), finals=np.array(fin, np.int16),
                        next_word=np.array(nxt, np.uint32))


def capture_train():
    """Three ModelManager.train_step calls on one fixed batch with the
    reference's test model/training configs (CPU, fp32), plus the checkpoint
    save_checkpoint writes afterwards."""
    import shutil
    import tempfile
    import torch
    import config as cfg
    from model import ModelManager
    tcfg = dict(cfg.test_training_config, device="cpu")
    torch.manual_seed(0)
    mm = ModelManager(cfg.test_model_config, tcfg)
    init = {k: v.detach().clone().numpy() for k, v in mm.model.state_dict().items()}
    g = torch.Generator().manual_seed(1)
    B = 8
    board = (torch.rand(B, 38, 5, 7, generator=g) > 0.8).float()
    glob = torch.rand(B, 42, generator=g)
    vis = torch.randint(0, 20, (B, 143), generator=g).float()
    pi = vis / vis.sum(1, keepdim=True)
    z = torch.randint(-1, 2, (B, 1), generator=g).float()
    losses = [mm.train_step(board, glob, pi, z) for _ in range(3)]
    final = {k: v.detach().clone().numpy() for k, v in mm.model.state_dict().items()}
    out = {"board": board.numpy(), "glob": glob.numpy(), "pi": pi.numpy(), "z": z.numpy(),
           "losses": np.array(losses, np.float64)}
    out.update({"init/" + k: v for k, v in init.items()})
    out.update({"final/" + k: v for k, v in final.items()})
    np.savez_compressed(os.path.join(OUT, "train.npz"), **out)
    d = tempfile.mkdtemp()
    try:
        mm.save_checkpoint(folder=d, filename="ck.pth.tar", iteration=7)
        shutil.copy(os.path.join(d, "ck.pth.tar"), os.path.join(OUT, "ref_ckpt_tiny.pth.tar"))
    finally:
        shutil.rmtree(d)


def main():
    parts = set(sys.argv[1:]) or {"mt", "env", "encoder", "scoring", "mcts", "greedy", "train"}
    he, pgs, mcts_mod = import_reference()
    import constants as C
    sorted_coords = list(C.sorted_coords)
    idx_of = {c: i for i, c in enumerate(sorted_coords)}
    if "mt" in parts:
        capture_mt()
    if parts & {"env", "encoder", "mcts"}:
        states = capture_env(he, pgs, idx_of)
        if "encoder" in parts:
            capture_encoder(he, pgs, states, sorted_coords, idx_of)
        if "mcts" in parts:
            capture_mcts(he, pgs, mcts_mod, states, sorted_coords, idx_of)
    if "scoring" in parts:
        capture_scoring(he, sorted_coords, idx_of)
    if "greedy" in parts:
        capture_greedy(he, pgs, idx_of)
    if "train" in parts:
        capture_train()
    for f in sorted(os.listdir(OUT)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(OUT, f)))


if __name__ == "__main__":
    main()
